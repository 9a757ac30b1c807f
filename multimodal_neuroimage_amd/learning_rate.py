"""Learning-rate handling of the training driver (learning_rate.py:18-169 of the reference).

`LrHandler(train_loader, **kwargs)` with `set_schedule(optimizer)` and
`schedule_check_and_update(optimizer)`, stepping once per iteration as the reference does:
  step      torch StepLR(step_size=lr_step, gamma=lr_gamma), only while lr > 1e-7
  SGDR      linear warm-up then cosine annealing with restarts (CosineAnnealingWarmUpRestarts,
            learning_rate.py:86-169): cycle length T_0 = 0.3 * total iterations, restart gamma 0.5
  OneCycle  torch OneCycleLR(max_lr = lr_init)
  CosAnn    torch CosineAnnealingLR(T_max = 100)
"""
import math

import torch
from torch.optim import lr_scheduler

FINAL_LR = 1e-7


class CosineAnnealingWarmUpRestarts(lr_scheduler.LRScheduler):
    """Warm-up from min_lr to max_lr over warmup_steps, cosine decay back to min_lr over the rest
    of the cycle; each restart multiplies the cycle length (minus warm-up) by cycle_mult and the
    peak by gamma.  Sequential stepping (the trainer never passes an epoch)."""

    def __init__(self, optimizer, first_cycle_steps, cycle_mult=1.0, max_lr=0.1, min_lr=0.001, warmup_steps=0,
                 gamma=1.0, last_epoch=-1):
        if warmup_steps >= first_cycle_steps:
            raise ValueError("warmup_steps must be shorter than the first cycle")
        self.first_cycle_steps, self.cycle_mult = first_cycle_steps, cycle_mult
        self.base_max_lr = self.max_lr = max_lr
        self.min_lr, self.warmup_steps, self.gamma = min_lr, warmup_steps, gamma
        self.cur_cycle_steps, self.cycle, self.step_in_cycle = first_cycle_steps, 0, last_epoch
        super().__init__(optimizer, last_epoch)
        for g in self.optimizer.param_groups:
            g["lr"] = min_lr
        self.base_lrs = [min_lr for _ in self.optimizer.param_groups]

    def _lr(self, base):
        s = self.step_in_cycle
        if s == -1:
            return base
        if s < self.warmup_steps:
            return base + (self.max_lr - base) * s / self.warmup_steps
        frac = (s - self.warmup_steps) / (self.cur_cycle_steps - self.warmup_steps)
        return base + (self.max_lr - base) * 0.5 * (1.0 + math.cos(math.pi * frac))

    def get_lr(self):
        return [self._lr(b) for b in self.base_lrs]

    def step(self, epoch=None):
        if epoch is not None:
            raise NotImplementedError("CosineAnnealingWarmUpRestarts: explicit epochs are not used by the trainer")
        if not hasattr(self, "cycle"):      # the base-class constructor's initial step
            return super().step()
        self.step_in_cycle += 1
        if self.step_in_cycle >= self.cur_cycle_steps:
            self.cycle += 1
            self.step_in_cycle -= self.cur_cycle_steps
            self.cur_cycle_steps = int((self.cur_cycle_steps - self.warmup_steps) * self.cycle_mult) + self.warmup_steps
        self.max_lr = self.base_max_lr * self.gamma ** self.cycle
        self.last_epoch += 1
        for g, lr in zip(self.optimizer.param_groups, self.get_lr()):
            g["lr"] = lr


class LrHandler:
    """Schedule selection and the per-iteration update of the reference's LrHandler."""

    def __init__(self, train_loader, **kwargs):
        self.kwargs = kwargs
        self.base_lr = kwargs.get("lr_init")
        self.lr_policy = kwargs.get("lr_policy")
        self.step_size = kwargs.get("lr_step")
        self.epoch = kwargs.get("nEpochs")
        self.num_iterations = len(train_loader)
        self.total_iterations = self.num_iterations * self.epoch
        self.gamma = 0.5 if self.lr_policy == "SGDR" else kwargs.get("lr_gamma")
        warm = kwargs.get("lr_warmup")
        self.warmup = int(self.total_iterations * 0.05) if warm is None else warm
        self.T_0 = int(0.3 * self.total_iterations)
        self.T_mult = kwargs.get("lr_T_mult") or 1
        self.final_lr = FINAL_LR
        self.schedule = None

    def set_lr(self, dict_lr):
        if self.base_lr is None:
            self.base_lr = dict_lr

    def set_schedule(self, optimizer):
        self.schedule = self.get_scheduler(optimizer)

    def get_scheduler(self, optimizer):
        if self.lr_policy == "step":
            return lr_scheduler.StepLR(optimizer, step_size=self.step_size, gamma=self.gamma)
        if self.lr_policy == "SGDR":
            for g in optimizer.param_groups:
                g["lr"] = 0
            return CosineAnnealingWarmUpRestarts(optimizer, first_cycle_steps=self.T_0, cycle_mult=self.T_mult,
                                                 max_lr=self.base_lr, min_lr=1e-9, warmup_steps=self.warmup,
                                                 gamma=self.gamma)
        if self.lr_policy == "OneCycle":
            return lr_scheduler.OneCycleLR(optimizer, max_lr=self.base_lr, steps_per_epoch=self.num_iterations,
                                           epochs=self.epoch)
        if self.lr_policy == "CosAnn":
            return lr_scheduler.CosineAnnealingLR(optimizer, T_max=100, eta_min=0)
        raise NotImplementedError(f"learning rate policy [{self.lr_policy}] is not implemented")

    def schedule_check_and_update(self, optimizer):
        """One scheduler step per iteration; the step policy stops at lr <= 1e-7."""
        if self.lr_policy == "step":
            if optimizer.param_groups[0]["lr"] > self.final_lr:
                self.schedule.step()
        else:
            self.schedule.step()
