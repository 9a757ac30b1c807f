"""Training driver with the reference's entry points (trainer.py:31-783), MI355X-native inside.

`Trainer(sets, **kwargs)`, `.training()`, `.testing()` keep the reference's constructor order,
method names and checkpoint schema so `main.py`'s `run_phase` / `test` can drive it unchanged
(SURVEY §2 L4, §8b).  What changes is the step internals:
  * one process per GPU, DDP over RCCL with a static graph (distributed.wrap_ddp) instead of
    DataParallel / find_unused_parameters;
  * no per-step host syncs: losses, NaN flags and per-subject logits stay on the device and are
    read back once per summary (the reference calls .item(), .isnan().sum() and .cpu() every
    step, trainer.py:548-563, 756-778);
  * validation / test predictions are gathered over ranks before the metrics (metrics.py);
  * checkpoints are written by rank 0 only, in the reference's schema (trainer.py:623-690);
  * the hot path computes in fp32 through the HIP kernels: `amp` keeps its GradScaler API but
    autocast is not entered (the kernels take fp32 operands; SURVEY §8d C3 is fp32).
Model zoo: the hot-path models of this build (SwinFusion, SwinTransformerV2,
Transformer_Net_Cross_Attention); other reference models raise NotImplementedError.
Datasets: `DataHandler.get_dataset()` returns a Dataset class built with **kwargs exposing the
reference protocol (`index_l`, `__getitem__` -> dict with the model inputs, 'subject' and the
target); the ABCD file readers are out of scope, so callers (and the tests) plug one
in the way the reference's own dataset registry does.
"""
import csv
import contextlib
import os
import warnings
from itertools import zip_longest

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, RandomSampler, Subset

from . import distributed as D
from . import model as M
from .learning_rate import LrHandler
from .metrics import classification_metrics, regression_metrics


@contextlib.contextmanager
def roctx_range(name):
    """A roctx range (torch.cuda.nvtx maps to roctx on ROCm) around a step phase, as the reference's
    torch.cuda.nvtx.range_push/pop pairs (trainer.py:373-430); a no-op cost when no profiler listens."""
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()

def reproducibility(**kwargs):
    """utils.py:134-142: seed torch (and its GPU generators) and numpy."""
    seed = kwargs.get("seed")
    torch.manual_seed(seed)
    if kwargs.get("cuda") and torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
    np.random.seed(seed)


class _ShardedSampler(torch.utils.data.Sampler):
    """DistributedSampler semantics over a Subset (distributed.ShardSampler)."""

    def __init__(self, n, env, shuffle, seed):
        self.inner = D.ShardSampler(n, env.rank, env.world, shuffle=shuffle, seed=seed)

    def set_epoch(self, epoch):
        self.inner.set_epoch(epoch)

    def __iter__(self):
        return iter(self.inner)

    def __len__(self):
        return len(self.inner)


class DataHandler:
    """Subject split + DataLoaders (dataloaders.py:17-182): random split by subject with numpy's
    seeded RNG (train_split / val_split), Subset per set, DistributedSampler semantics when
    distributed else RandomSampler, drop_last, pinned batches."""

    datasets = {}   # dataset_name -> Dataset class (the reference's get_dataset registry)

    def __init__(self, test=False, **kwargs):
        self.kwargs = kwargs
        self.dataset_name = kwargs.get("dataset_name")
        self.step = kwargs.get("step")
        self.seed = kwargs.get("seed")
        self.env = kwargs.get("env") or D.DistEnv()

    def get_dataset(self):
        if self.dataset_name not in self.datasets:
            raise NotImplementedError(f"dataset {self.dataset_name!r}: register a Dataset class in "
                                      "DataHandler.datasets (the ABCD readers are out of scope)")
        return self.datasets[self.dataset_name]

    def determine_split_randomly(self, index_l, **kwargs):
        S = len(np.unique([x[0] for x in index_l]))
        n_train = int(S * kwargs.get("train_split"))
        n_val = int(S * kwargs.get("val_split"))
        s_train = np.random.choice(S, n_train, replace=False)
        rest = np.setdiff1d(np.arange(S), s_train)
        s_val = np.random.choice(rest, n_val, replace=False)
        s_test = np.setdiff1d(np.arange(S), np.concatenate([s_train, s_val]))
        return self.convert_subject_list_to_idx_list(s_train, s_val, s_test, index_l)

    @staticmethod
    def convert_subject_list_to_idx_list(train_names, val_names, test_names, subj_list):
        ids = np.array([str(x[0]) for x in subj_list])
        pick = lambda names: np.where(np.isin(ids, [str(n) for n in names]))[0].tolist()
        return pick(train_names), pick(val_names), pick(test_names)

    def _loader(self, ds, shuffle, sampler=None):
        if sampler is None:
            if self.env.enabled:
                sampler = _ShardedSampler(len(ds), self.env, shuffle, self.seed or 0)
            else:
                sampler = RandomSampler(ds)
        return DataLoader(ds, batch_size=self.kwargs.get("batch_size"), num_workers=self.kwargs.get("workers") or 0,
                          drop_last=True, pin_memory=torch.cuda.is_available(), sampler=sampler,
                          persistent_workers=bool(self.kwargs.get("workers")))

    def create_dataloaders(self):
        reproducibility(**self.kwargs)
        cls = self.get_dataset()
        train_ds, eval_ds = cls(**self.kwargs), cls(**self.kwargs)
        eval_ds.augment = None
        self.subject_list = train_ds.index_l
        tr, va, te = self.determine_split_randomly(self.subject_list, **self.kwargs)
        samplers = self.kwargs.get("samplers") or {}
        train = self._loader(Subset(train_ds, tr), True, samplers.get("train"))
        val = self._loader(Subset(eval_ds, va), False, samplers.get("val"))
        test = self._loader(Subset(eval_ds, te), False, samplers.get("test")) if self.step == "4" else None
        return train, val, test


class Writer:
    """Loss / metric bookkeeping (loss_writer.py:15-212) minus TensorBoard and wandb: running loss
    values per set (device scalars, read back once per summary), per-subject predictions, CSV
    history in <experiment_folder>/history/full_scores.csv on rank 0."""

    def __init__(self, sets, val_threshold, **kwargs):
        self.kwargs = kwargs
        self.sets, self.val_threshold = sets, val_threshold
        self.env = kwargs.get("env") or D.DistEnv()
        self.fine_tune_task = kwargs.get("fine_tune_task")
        self.experiment_folder = kwargs.get("experiment_folder")
        self.experiment_title = kwargs.get("experiment_title")
        self.running_mean_size = int(kwargs.get("running_mean_size") or 5000)
        self.total_train_steps = 0
        self.eval_iter = 0
        self.current_metrics = {}
        self.loss_names = ["regression" if self.fine_tune_task == "regression" else "binary_classification", "total"]
        self.values = {(n, s): [] for n in self.loss_names for s in sets}
        self.history = {(n, s): [] for n in self.loss_names for s in sets}
        self.records = []            # (mode, subject ids (device), scores (device), truth (device))

    def write_losses(self, loss_dict, set):
        for name, v in loss_dict.items():
            vals = self.values[(name, set)]
            vals.append(v.detach())
            if set == "train" and len(vals) > self.running_mean_size:
                del vals[:-self.running_mean_size]

    def loss_summary(self, lr):
        for (name, s), vals in self.values.items():
            if not vals:
                continue
            t = torch.stack([v.float() for v in vals]).mean()
            if self.env.enabled:      # mean over ranks
                dist.all_reduce(t)
                t /= self.env.world
            score = float(t.item())
            self.history[(name, s)].append(score)
            setattr(self, f"{name}_{s}_loss_history", self.history[(name, s)])
            print(f"{name}_{s}: {score}")
            # as the reference: validation values accumulate over epochs (loss_writer.py:147-155
            # trims only the training list to the running window)

    def record(self, mode, subjects, scores, truth):
        self.records.append((mode, subjects.detach(), scores.detach().float().reshape(-1), truth.detach().float()
                             .reshape(-1)))

    def _gather(self):
        """All ranks' (mode, subject, score, truth) rows on every rank."""
        modes = {m: i for i, m in enumerate(["train", "val", "test"])}
        if not self.records:
            rows = torch.zeros(0, 4, dtype=torch.float64)
        else:
            rows = torch.cat([torch.stack([torch.full_like(sc, modes[m], dtype=torch.float64),
                                           sb.to(sc.device).double(), sc.double(), tr.to(sc.device).double()], 1)
                              for m, sb, sc, tr in self.records]).cpu()
        if self.env.enabled:
            dev = self.env.device
            n = torch.tensor([rows.shape[0]], device=dev)
            sizes = [torch.zeros_like(n) for _ in range(self.env.world)]
            dist.all_gather(sizes, n)
            cap = int(max(s.item() for s in sizes))
            pad = torch.zeros(cap, 4, dtype=torch.float64, device=dev)
            pad[:rows.shape[0]] = rows.to(dev)
            parts = [torch.zeros_like(pad) for _ in range(self.env.world)]
            dist.all_gather(parts, pad)
            rows = torch.cat([p[:int(s.item())] for p, s in zip(parts, sizes)]).cpu()
        inv = {i: m for m, i in modes.items()}
        return [(inv[int(r[0])], int(r[1]), float(r[2]), float(r[3])) for r in rows]

    def accuracy_summary(self, mid_epoch):
        subj = {}
        for mode, s, score, truth in self._gather():
            d = subj.setdefault(s, {"scores": [], "truth": truth, "mode": mode})
            d["scores"].append(score)
        preds = {s: [] for s in self.sets}
        truths = {s: [] for s in self.sets}
        for s, d in subj.items():
            sc = torch.tensor(d["scores"])
            if self.fine_tune_task == "binary_classification":
                sc = torch.sigmoid(sc)
            if d["mode"] in preds:
                preds[d["mode"]].append(float(sc.mean()))
                truths[d["mode"]].append(d["truth"])
        metrics = {}
        for name in self.sets:
            if not preds[name]:
                continue
            if self.fine_tune_task == "regression":
                metrics.update(regression_metrics(truths[name], preds[name], name))
            else:
                metrics.update(classification_metrics(truths[name], preds[name], name, self.val_threshold))
        self.current_metrics = metrics
        for k, v in metrics.items():
            getattr(self, k, None) is None and setattr(self, k, [])
            getattr(self, k).append(v)
            print(f"{k}: {v}")
        self.eval_iter += 1
        self.records = [r for r in self.records if r[0] == "train"] if mid_epoch else []

    def save_history_to_csv(self):
        if self.env.rank != 0 or not self.experiment_folder:
            return
        path = os.path.join(self.experiment_folder, "history")
        os.makedirs(path, exist_ok=True)
        cols = {f"{n}_{s}_loss_history": h for (n, s), h in self.history.items()}
        cols.update({k: getattr(self, k) for k in self.current_metrics})
        names = sorted(cols)
        with open(os.path.join(path, "full_scores.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(names)
            w.writerows(zip_longest(*[cols[n] for n in names], fillvalue=""))


class Trainer:
    """Training / validation / test driver (trainer.py:31-783)."""

    def __init__(self, sets, **kwargs):
        self.register_args(**kwargs)
        self.env = kwargs.get("env") or D.init_from_env(use_cuda=bool(kwargs.get("cuda", True)))
        self.kwargs["env"] = self.env
        self.distributed = self.env.enabled
        self.rank = self.env.rank
        self.device = self.env.device
        self.eval_iter = 0
        self.best_loss = 100000
        self.best_AUROC = 0
        self.best_ACC = 0
        self.val_threshold = 0
        self.st_epoch = 1
        self.recent_pth = None
        self.state_dict = None
        self.mode = "train"
        self.train_loader, self.val_loader, self.test_loader = DataHandler(**self.kwargs).create_dataloaders()
        self.lr_handler = LrHandler(self.train_loader, **self.kwargs)
        self.create_model()
        self.load_model_checkpoint()
        self.set_model_device()
        self.create_optimizer()
        self.lr_handler.set_schedule(self.optimizer)
        self.scaler = torch.amp.GradScaler("cuda", enabled=False)   # fp32 HIP path: scaling is a no-op
        self.load_optim_checkpoint()
        self.writer = Writer(sets, self.val_threshold, **self.kwargs)
        self.sets = sets
        self.nan_flag = torch.zeros((), device=self.device, dtype=torch.int32)

    # ---- construction ------------------------------------------------------------------
    def register_args(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)
        self.kwargs = dict(kwargs)

    def create_model(self):
        task = (self.kwargs.get("task") or "").lower()
        ds = self.kwargs.get("dataset_name")
        if task == "swinfusion" or ds == "struct":
            self.model = M.SwinFusion(**self.kwargs)
        elif (task in ("vit", "test") and self.kwargs.get("VIT_name") == "swinv2") or ds in ("DTI", "sMRI", "DTI+sMRI"):
            self.model = M.SwinTransformerV2(**self.kwargs)
        elif task in ("lowfreqbert", "test") and self.kwargs.get("fmri_multimodality_type") == "cross_attention":
            self.model = M.Transformer_Net_Cross_Attention(**self.kwargs)
        else:
            raise NotImplementedError(f"task {task!r} / dataset {ds!r}: not a hot-path model of this build")

    def _net(self):
        return self.model.module if hasattr(self.model, "module") else self.model

    def set_model_device(self):
        self.model = D.wrap_ddp(self.model.to(self.device), self.env)

    def create_optimizer(self):
        opt = getattr(torch.optim, self.kwargs.get("optim"))
        self.optimizer = opt(self.model.parameters(), lr=self.lr_handler.base_lr,
                             weight_decay=self.kwargs.get("weight_decay"))

    # ---- checkpoints (trainer.py:107-162, 623-690) --------------------------------------------
    def _sort_pth_files(self, folder):
        files = [(f, os.path.getctime(os.path.join(folder, f))) for f in os.listdir(folder) if f.endswith(".pth")]
        return sorted(files, key=lambda x: x[1], reverse=True)

    def load_model_checkpoint(self):
        folder = self.kwargs.get("experiment_folder")
        pths = self._sort_pth_files(folder) if folder and os.path.isdir(folder) else []
        weights = self.kwargs.get("loaded_model_weights_path")
        if pths:
            self.recent_pth = pths[0][0]
            path = os.path.join(folder, self.recent_pth)
        elif weights:
            path = weights
        else:
            return
        self.state_dict = torch.load(path, map_location="cpu", weights_only=True)
        self.model.load_partial_state_dict(self.state_dict["model_state_dict"], load_cls_embedding=True)
        self.model.loaded_model_weights_path = path

    def load_optim_checkpoint(self):
        if self.recent_pth:
            self.optimizer.load_state_dict(self.state_dict["optimizer_state_dict"])
            if self.state_dict.get("schedule_state_dict") is not None:
                self.lr_handler.schedule.load_state_dict(self.state_dict["schedule_state_dict"])
            if self.state_dict.get("amp_state"):
                self.scaler.load_state_dict(self.state_dict["amp_state"])
            self.st_epoch = int(self.state_dict["epoch"]) + 1
            self.best_loss = self.state_dict["loss_value"]
        elif self.state_dict and "val_threshold" in self.state_dict:
            self.val_threshold = self.state_dict["val_threshold"]

    def save_checkpoint_(self, epoch, batch_idx, scaler):
        if self.rank != 0:
            return
        loss = self.get_last_loss()
        val_acc, val_auroc, val_thr = self.get_last_ACC(), self.get_last_AUROC(), self.get_last_val_threshold()
        title = f"{self.kwargs.get('experiment_title')}_epoch_{int(epoch)}"
        folder = self.kwargs.get("experiment_folder")
        os.makedirs(folder, exist_ok=True)
        ckpt = {"model_state_dict": self._net().state_dict(), "optimizer_state_dict": self.optimizer.state_dict(),
                "epoch": epoch, "loss_value": loss, "amp_state": scaler.state_dict()}
        if val_auroc is not None:
            ckpt["val_AUROC"] = val_auroc
        if val_thr is not None:
            ckpt["val_threshold"] = val_thr
        if self.lr_handler.schedule is not None:
            ckpt["schedule_state_dict"] = self.lr_handler.schedule.state_dict()
            ckpt["lr"] = self.optimizer.param_groups[0]["lr"]
        if getattr(self._net(), "loaded_model_weights_path", None):
            ckpt["loaded_model_weights_path"] = self._net().loaded_model_weights_path
        name = None
        if val_auroc is not None:
            if self.best_AUROC < val_auroc:
                self.best_AUROC = val_auroc
                name = f"{title}_BEST_val_AUROC.pth"
                self.best_ACC = max(self.best_ACC, val_acc)
            elif self.best_ACC < val_acc:
                self.best_ACC = val_acc
                name = f"{title}_BEST_val_ACC.pth"
        elif self.best_loss > loss:
            self.best_loss = loss
            name = f"{title}_BEST_val_loss.pth"
        if name:
            torch.save(ckpt, os.path.join(folder, name))
        return name

    def get_last_loss(self):
        if self.kwargs.get("fine_tune_task") == "regression":
            return self.writer.val_MAE[-1]
        return self.writer.total_val_loss_history[-1]

    def get_last_AUROC(self):
        return self.writer.val_AUROC[-1] if hasattr(self.writer, "val_AUROC") else None

    def get_last_ACC(self):
        return self.writer.val_Balanced_Accuracy[-1] if hasattr(self.writer, "val_Balanced_Accuracy") else None

    def get_last_val_threshold(self):
        return self.writer.val_best_threshold[-1] if hasattr(self.writer, "val_best_threshold") else None

    # ---- loops ----------------------------------------------------------------------------
    def training(self):
        n_epochs = 1 if self.kwargs.get("profiling") else self.kwargs.get("nEpochs")
        for epoch in range(self.st_epoch, n_epochs + 1):
            self.train_epoch(epoch)
            self.eval_epoch("val")
            self.writer.loss_summary(lr=self.optimizer.param_groups[0]["lr"])
            self.writer.accuracy_summary(mid_epoch=False)
            self.writer.save_history_to_csv()
            self.save_checkpoint_(epoch, len(self.train_loader), self.scaler)
        return self.best_AUROC, self.best_loss

    def train_epoch(self, epoch):
        sampler = getattr(self.train_loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        self.train()
        acc = int(self.kwargs.get("accumulation_steps") or 1)
        for batch_idx, input_dict in enumerate(self.train_loader):
            self.writer.total_train_steps += 1
            # roctx ranges at the reference's NVTX points (trainer.py:373-430): rocprofv3
            # --marker-trace lines its kernel trace up with them
            with roctx_range("training step"):
                self.optimizer.zero_grad()
                with roctx_range("forward"):
                    loss_dict, loss = self.forward_pass(input_dict)
                with roctx_range("backward"):
                    (loss / acc).backward()
                if (batch_idx + 1) % acc == 0:
                    if self.kwargs.get("gradient_clipping"):
                        with roctx_range("clip"):
                            torch.nn.utils.clip_grad_norm_(self.model.parameters(),
                                                           max_norm=self.kwargs.get("clip_max_norm"))
                    with roctx_range("optimize"):
                        self.optimizer.step()
            self.lr_handler.schedule_check_and_update(self.optimizer)
            self.writer.write_losses(loss_dict, set="train")
            if self.kwargs.get("profiling") and batch_idx == 10:
                break
        self.check_nans(f"epoch {epoch}")

    def check_nans(self, where):
        """One device read per epoch of the NaN flag the steps OR into (the reference checks every
        step with a host sync and warns, trainer.py:548-555); warn the same way, then reset."""
        if int(self.nan_flag.item()):
            warnings.warn('found nans in computation')
            print(f'at {where}: a training loss was NaN')
            self.nan_flag.zero_()

    def eval_epoch(self, set):
        loader = self.val_loader if set == "val" else self.test_loader
        self.eval(set)
        with torch.no_grad():
            for batch_idx, input_dict in enumerate(loader):
                loss_dict, _ = self.forward_pass(input_dict)
                self.writer.write_losses(loss_dict, set=set)
                if self.kwargs.get("profiling") and batch_idx == 10:
                    break

    def testing(self):
        self.eval_epoch("test")
        self.writer.loss_summary(lr=0)
        self.writer.accuracy_summary(mid_epoch=False)

    def train(self):
        self.mode = "train"
        self.model.train()

    def eval(self, set):
        self.mode = set
        self.model.eval()

    # ---- one step (trainer.py:475-567, 739-778) ---------------------------------------------
    def _inputs(self, d):
        ds = self.kwargs.get("dataset_name")
        if ds == "struct":
            return d["smri"], d["dti"]
        if ds == "DTI":
            return (d["dti"],)
        if ds == "sMRI":
            return (d["smri"],)
        if ds == "DTI+sMRI":
            return (d["struct"],)
        if self.kwargs.get("fmri_multimodality_type") == "cross_attention":
            return d["fmri_lowfreq_sequence"], d["fmri_ultralowfreq_sequence"]
        raise NotImplementedError(f"dataset {ds!r}: no input routing in this build")

    def forward_pass(self, input_dict):
        d = {k: (v.to(self.device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in input_dict.items()}
        inputs = [x.float() for x in self._inputs(d)]
        output_dict = self.model(*inputs)
        loss_dict, loss = self.aggregate_losses(d, output_dict)
        self.compute_accuracy(d, output_dict)
        return loss_dict, loss

    def aggregate_losses(self, input_dict, output_dict):
        task = self.kwargs.get("fine_tune_task")
        target = input_dict[self.kwargs.get("target")]
        out = output_dict[task].squeeze()
        if task == "regression":
            loss = torch.nn.functional.l1_loss(out, target.squeeze())
        else:
            loss = torch.nn.functional.binary_cross_entropy_with_logits(out, target.squeeze().float())
        self.nan_flag |= torch.isnan(loss).int()       # checked at summaries, no per-step sync
        name = "regression" if task == "regression" else "binary_classification"
        return {name: loss.detach(), "total": loss.detach()}, loss

    def compute_accuracy(self, input_dict, output_dict):
        task = self.kwargs.get("fine_tune_task")
        self.writer.record(self.mode, input_dict["subject"], output_dict[task], input_dict[self.kwargs.get("target")])
