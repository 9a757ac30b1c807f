"""Import the reference's hot-path modules in the BUILD container only (never on the GPU box).

Used solely by tests/golden/make_golden.py to produce the committed fixtures.  Two shims,
neither of which changes arithmetic:
  * a 3-symbol `timm.models.layers` stub (DropPath, to_2tuple, trunc_normal_), removed again
    before `import model` because transformers probes timm's __spec__;
  * Tensor.get_device() returning 'cpu' instead of -1 (swin_v2_module.py:154 etc.).
"""
import argparse
import ast
import os
import sys
import types

import torch
import torch.nn as nn

REF = "/root/reference"


def _timm_stub():
    layers = types.ModuleType("timm.models.layers")

    class DropPath(nn.Module):
        def __init__(self, p=0.0):
            super().__init__()
            self.drop_prob = p

        def forward(self, x):
            if self.drop_prob == 0.0 or not self.training:
                return x
            keep = 1 - self.drop_prob
            mask = x.new_empty((x.shape[0],) + (1,) * (x.ndim - 1)).bernoulli_(keep)
            return x * mask / keep

    layers.DropPath = DropPath
    layers.trunc_normal_ = nn.init.trunc_normal_
    layers.to_2tuple = lambda x: tuple(x) if isinstance(x, (list, tuple)) else (x, x)
    models = types.ModuleType("timm.models")
    models.layers = layers
    timm = types.ModuleType("timm")
    timm.models = models
    return {"timm": timm, "timm.models": models, "timm.models.layers": layers}


_loaded = {}


def load():
    """Return dict of reference modules: swin_v2, swinfusion, mha, crossmodal, pe, model."""
    if _loaded:
        return _loaded
    if not os.path.isdir(REF):
        raise RuntimeError("reference not present (fixtures are generated in the build container only)")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    stub = _timm_stub()
    sys.modules.update(stub)
    import modules.swin_v2_module as swin_v2
    import modules.swinfusion_module as swinfusion
    import modules.multihead_attention as mha
    import modules.crossmodal_transformer as crossmodal
    import modules.position_embedding as pe
    for k in stub:
        del sys.modules[k]
    gd = torch.Tensor.get_device
    torch.Tensor.get_device = lambda self: "cpu" if gd(self) == -1 else gd(self)
    import model as M
    _loaded.update(swin_v2=swin_v2, swinfusion=swinfusion, mha=mha, crossmodal=crossmodal, pe=pe, model=M)
    return _loaded


def default_kwargs(step, argv=()):
    """kwargs the reference Trainer passes to model constructors for phase `step`
    (main.get_arguments + utils.sort_args), without importing main.py (it imports optuna)."""
    src = open(os.path.join(REF, "main.py")).read()
    fn = [n for n in ast.parse(src).body if isinstance(n, ast.FunctionDef) and n.name == "get_arguments"][0]
    ns = {"argparse": argparse, "os": os}
    exec(compile(ast.Module([fn], []), "main.py", "exec"), ns)
    old = sys.argv
    sys.argv = ["main.py", "--step", step, *argv]
    try:
        a = vars(ns["get_arguments"]("/tmp"))
    finally:
        sys.argv = old
    kw = {k: v for k, v in a.items() if "phase" not in k}
    kw.update({k.replace("_phase" + step, ""): v for k, v in a.items() if "phase" + step in k})
    return kw
