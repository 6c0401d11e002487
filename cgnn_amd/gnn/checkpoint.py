"""GNN-track checkpoint format (new; the reference has no model checkpoints).

One ``.safetensors`` file per trainer (no pickle: loading executes nothing from
the file):

* tensors -- the trainer's parameters and optimizer state under stable names
  (``model.<state_dict key>``, ``opt.<param index>.{exp_avg,exp_avg_sq,step}``
  for PyTorch-optimizer trainers; ``params`` / ``adam_m`` / ``adam_v`` /
  ``adam_step`` for the fused GCN trainer's flat buffers);
* metadata -- ``format`` (``cgnn_amd.gnn/1``), ``trainer`` (class name),
  ``epoch``, and ``config`` (JSON of the constructor arguments the caller
  passes) so a run can be rebuilt and resumed bit-for-bit on one device.

Trainers implement ``state_tensors() -> dict`` and ``load_state_tensors(dict)``
or are handled here through their ``model`` / ``opt`` attributes.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Optional

import torch

from ..utils.checkpoint import load_tensors, save_tensors

FORMAT = "cgnn_amd.gnn/1"


def module_optimizer_tensors(model: torch.nn.Module, opt: torch.optim.Optimizer) -> Dict[str, torch.Tensor]:
    t = {"model." + k: v for k, v in model.state_dict().items()}
    for i, p in enumerate(model.parameters()):
        st = opt.state.get(p, {})
        for k in ("exp_avg", "exp_avg_sq", "step"):
            if k in st:
                v = st[k]
                t["opt.%d.%s" % (i, k)] = v.reshape(-1) if k == "step" else v
    return t


def load_module_optimizer_tensors(model: torch.nn.Module, opt: torch.optim.Optimizer, t: Dict[str, torch.Tensor]):
    model.load_state_dict({k[6:]: v for k, v in t.items() if k.startswith("model.")})
    capturable = any(g.get("capturable", False) for g in opt.param_groups)
    for i, p in enumerate(model.parameters()):
        if "opt.%d.exp_avg" % i not in t:
            continue
        st = opt.state[p]
        st["exp_avg"] = t["opt.%d.exp_avg" % i].to(p.device).clone()
        st["exp_avg_sq"] = t["opt.%d.exp_avg_sq" % i].to(p.device).clone()
        step = t["opt.%d.step" % i].to(torch.float32).reshape(()).clone()
        st["step"] = step.to(p.device) if capturable else step


def trainer_tensors(tr) -> Dict[str, torch.Tensor]:
    if hasattr(tr, "state_tensors"):
        return tr.state_tensors()
    return module_optimizer_tensors(tr.model, tr.opt)


def save_trainer(tr, path: str, config: Optional[Dict[str, Any]] = None):
    """Write ``tr``'s parameters + optimizer state (rank 0 writes under DP: the
    replicas are identical)."""
    meta = {"format": FORMAT, "trainer": type(tr).__name__, "epoch": str(int(getattr(tr, "epoch", 0))),
            "config": json.dumps(config or {})}
    save_tensors(path, trainer_tensors(tr), meta)


def read_metadata(path: str) -> Dict[str, Any]:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        meta = dict(f.metadata() or {})
    if meta.get("format") != FORMAT:
        raise ValueError("%s is not a %s checkpoint" % (path, FORMAT))
    meta["config"] = json.loads(meta.get("config", "{}"))
    return meta


def load_trainer(tr, path: str) -> Dict[str, Any]:
    """Restore ``tr`` (constructed with the same shapes) from ``path``; returns the metadata."""
    meta = read_metadata(path)
    if meta["trainer"] != type(tr).__name__:
        raise ValueError("checkpoint holds a %s, not a %s" % (meta["trainer"], type(tr).__name__))
    t = load_tensors(path)
    if hasattr(tr, "load_state_tensors"):
        tr.load_state_tensors(t)
    else:
        load_module_optimizer_tensors(tr.model, tr.opt, t)
    tr.epoch = int(meta["epoch"])
    return meta
