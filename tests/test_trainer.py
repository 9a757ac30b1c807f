"""Trainer plumbing on CPU against the reference Trainer's own run (tests/golden/trainer.json,
made by tests/golden/make_trainer_golden.py): subject split, validation metrics from the
recorded logits, learning-rate schedule."""
import json
import os

import numpy as np
import pytest
import torch

from multimodal_neuroimage_amd import learning_rate as LR
from multimodal_neuroimage_amd.metrics import classification_metrics
from multimodal_neuroimage_amd.trainer import DataHandler, reproducibility

GOLD = os.path.join(os.path.dirname(__file__), "golden", "trainer.json")


@pytest.fixture(scope="module")
def gold():
    return json.load(open(GOLD))


def test_subject_split_matches_reference(gold):
    kw = dict(gold["kwargs"])
    reproducibility(**{**kw, "cuda": False})
    index_l = [(i, f"SUBJ{i:03d}") for i in range(gold["n_subjects"])]
    tr, va, te = DataHandler(**kw).determine_split_randomly(index_l, **kw)
    assert tr == gold["split"]["train"] and va == gold["split"]["val"]
    assert sorted(tr + va + te) == list(range(gold["n_subjects"]))


def test_val_metrics_from_reference_logits(gold):
    """The metric code on the reference run's last-epoch validation logits reproduces its
    reported metrics (per-subject mean of sigmoid, sklearn as the reference calls it)."""
    n_val = len(gold["split"]["val"])
    last = gold["val"][-(n_val // gold["kwargs"]["batch_size"]):]
    subj, truth = {}, {}
    labels = {i: float((i * 7 + 3) % 5 < 2) for i in range(gold["n_subjects"])}   # make_trainer_golden.label
    for b in last:
        for s, z in zip(b["subjects"], b["logits"]):
            subj.setdefault(s, []).append(z)
            truth[s] = labels[s]
    keys = list(subj)
    pred = [float(torch.sigmoid(torch.tensor(subj[k])).mean()) for k in keys]
    got = classification_metrics([truth[k] for k in keys], pred, "val", 0)
    for k, v in gold["metrics"].items():
        assert got[k] == pytest.approx(v, rel=1e-6, abs=1e-9), k


def test_step_lr_policy_matches_reference_lr(gold):
    kw = gold["kwargs"]
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=kw["lr_init"], weight_decay=kw["weight_decay"])

    class _L:
        def __len__(self):
            return len(gold["train"]) // kw["nEpochs"]

    h = LR.LrHandler(_L(), **kw)
    h.set_schedule(opt)
    lrs = []
    for _ in gold["train"]:
        lrs.append(opt.param_groups[0]["lr"])
        h.schedule_check_and_update(opt)
    assert lrs == pytest.approx([t["lr"] for t in gold["train"]], rel=1e-12)


def test_sgdr_warmup_then_cosine_restarts():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=1e-3)

    class _L:
        def __len__(self):
            return 100

    h = LR.LrHandler(_L(), lr_init=1e-3, lr_policy="SGDR", lr_step=10, nEpochs=2, lr_gamma=0.9, lr_warmup=10)
    h.set_schedule(opt)
    seen = []
    for _ in range(200):
        h.schedule_check_and_update(opt)
        seen.append(opt.param_groups[0]["lr"])
    T0 = int(0.3 * 200)
    assert seen[9] == pytest.approx(1e-3, rel=1e-6)          # end of warm-up: the peak
    assert max(seen[:T0]) == pytest.approx(1e-3, rel=1e-6)
    assert seen[T0 - 2] < 1e-5                                  # annealed towards min_lr
    assert max(seen[T0:2 * T0]) == pytest.approx(0.5e-3, rel=1e-6)   # restart peak x gamma 0.5
