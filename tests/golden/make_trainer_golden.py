"""Config-1 plumbing fixture: run the REFERENCE's own Trainer for one
epoch of SwinFusion on synthetic 84x84 sMRI/DTI pairs on CPU and record what the build's
Trainer must reproduce: the batch order it drew, the per-step training loss, the learning rate,
the validation logits and the validation metrics.

Build container only (the reference never travels to the GPU box):
    python tests/golden/make_trainer_golden.py
Writes tests/golden/trainer.json (a few hundred numbers).  Stubs (no arithmetic): wandb, tensorboard, torchvision,
nibabel, torchaudio, nitime, skimage are import-only no-ops; the timm DropPath stub is the
identity (drop_path forced to 0: the SwinFusion head hard-codes drop_path_rate 0.1,
model.py:1188, which is RNG-dependent and parity-unpinned); DataHandler.get_dataset returns a
synthetic Dataset; convert_subject_list_to_idx_list compares as strings (dataloaders.py:151-156
returns empty splits under numpy 2.x).  Parameters: tests/golden/recipe.py.
"""
import importlib.machinery
import json
import os
import sys
import tempfile
import types

import numpy as np
import scipy.stats
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import recipe  # noqa: E402
import refload  # noqa: E402

N_SUBJECTS = 40
IMG = 84
BATCH = 2


def volume(kind, i):
    """The synthetic subject volumes (the build test regenerates them the same way)."""
    return recipe.randn(1000 * (1 if kind == "smri" else 2) + i, (IMG, IMG))


def label(i):
    return float((i * 7 + 3) % 5 < 2)


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_stubs():
    class _Nop:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return lambda *a, **k: None

    _stub("wandb", init=lambda *a, **k: None, watch=lambda *a, **k: None, log=lambda *a, **k: None)
    _stub("torch.utils.tensorboard", SummaryWriter=_Nop)
    tv = _stub("torchvision")
    tv.models = _stub("torchvision.models")
    _stub("nibabel")
    ta = _stub("torchaudio")
    ta.functional = _stub("torchaudio.functional")
    nt = _stub("nitime")
    nt.timeseries = _stub("nitime.timeseries", TimeSeries=_Nop)
    nt.analysis = _stub("nitime.analysis", SpectralAnalyzer=_Nop, FilterAnalyzer=_Nop, NormalizationAnalyzer=_Nop)
    sk = _stub("skimage")
    sk.transform = _stub("skimage.transform", rescale=None, resize=None)


class SyntheticStruct(torch.utils.data.Dataset):
    """ABCD_struct stand-in (datasets.py:479-545): same item keys, the same z-score + .half()
    rounding; handed over as float32 (AMP is off on CPU and the fp32 model rejects fp16 input)."""

    def __init__(self, **kwargs):
        self.target = kwargs.get("target")
        self.index_l = [(i, f"SUBJ{i:03d}", None, None, torch.tensor(label(i))) for i in range(N_SUBJECTS)]
        self.augment = None

    def __len__(self):
        return len(self.index_l)

    def get_input_shape(self):
        return (IMG, IMG)

    def __getitem__(self, index):
        subj, name, _, _, target = self.index_l[index]
        smri = torch.Tensor(scipy.stats.zscore(volume("smri", subj), axis=None)).half().float()
        dti = torch.Tensor(scipy.stats.zscore(volume("dti", subj), axis=None)).half().float()
        return {"smri": smri, "dti": dti, "subject": subj, "subject_name": name, self.target: target}


def main():
    torch.set_num_threads(8)
    R = refload.load()       # modules + model.py first (transformers probes the stubbed packages)
    install_stubs()
    # the stubbed DropPath: identity (drop_path forced to 0)
    for mod in (R["swin_v2"], R["swinfusion"]):
        if hasattr(mod, "DropPath"):
            mod.DropPath.forward = lambda self, x: x
    sys.path.insert(0, refload.REF)
    import trainer as T
    import data_preprocess_and_load.dataloaders as DL

    DL.DataHandler.get_dataset = lambda self: SyntheticStruct

    def to_idx(self, train_names, val_names, test_names, subj_list):
        ids = np.array([str(x[0]) for x in subj_list])
        pick = lambda names: np.where(np.isin(ids, [str(n) for n in names]))[0].tolist()
        return pick(train_names), pick(val_names), pick(test_names)

    DL.DataHandler.convert_subject_list_to_idx_list = to_idx

    tmp = tempfile.mkdtemp()
    os.makedirs(os.path.join(tmp, "splits"), exist_ok=True)
    kw = refload.default_kwargs("6", ["--dataset_name", "struct"])
    kw.update(cuda=False, workers=0, batch_size=BATCH, nEpochs=2, base_path=tmp, experiment_folder=tmp,
              experiment_title="c1", log_dir=os.path.join(tmp, "runs"), wandb_mode="disabled", distributed=False,
              gpu=None, rank=0, amp=True, loaded_model_weights_path=None, model_weights_path=None)
    tr = T.Trainer(sets=["train", "val"], **kw)
    net = tr.model.module if hasattr(tr.model, "module") else tr.model
    recipe.fill_params(net)

    log = {"train": [], "val": []}
    last = {}
    orig_acc = tr.compute_accuracy

    def compute_accuracy(input_dict, output_dict):
        # the per-subject logits the writer accumulates (trainer.py:756-778)
        last["logits"] = [float(v) for v in output_dict[kw["fine_tune_task"]].detach().reshape(-1)]
        return orig_acc(input_dict, output_dict)

    orig = tr.forward_pass

    def forward_pass(input_dict):
        loss_dict, loss = orig(input_dict)
        log[tr.mode].append(dict(subjects=[int(s) for s in input_dict["subject"]], loss=float(loss_dict["total"]),
                                 lr=float(tr.optimizer.param_groups[0]["lr"]), logits=last.pop("logits")))
        return loss_dict, loss

    tr.compute_accuracy = compute_accuracy
    tr.forward_pass = forward_pass
    tr.training()
    w = tr.writer
    metrics = {k: float(getattr(w, k)[-1]) for k in dir(w)
               if k.startswith("val_") and isinstance(getattr(w, k), list) and getattr(w, k)
               and isinstance(getattr(w, k)[-1], (float, np.floating, int))}
    split = dict(train=sorted({s for st in log["train"] for s in st["subjects"]}),
                 val=sorted({s for st in log["val"] for s in st["subjects"]}))
    meta = dict(kwargs={k: v for k, v in kw.items() if isinstance(v, (str, int, float, bool, type(None)))},
                n_subjects=N_SUBJECTS, img=IMG, params=recipe.param_signature(net), train=log["train"], val=log["val"],
                split=split, metrics=metrics)
    out = os.path.join(HERE, "trainer.json")
    with open(out, "w") as f:
        json.dump(meta, f, indent=1, default=lambda o: list(o) if isinstance(o, tuple) else str(o))
    print(f"wrote {out}: {len(log['train'])} train steps, {len(log['val'])} val batches, metrics {metrics}")


if __name__ == "__main__":
    main()
