"""Fused Adam over every parameter of a group in one HIP launch.

The reference trains with `optim.Adam(net.parameters(), lr=lr,
weight_decay=5e-4)` (train_mobilenetV3_ecagai.py:564) and calls
`optimizer.step()` once per batch (:588).  `Adam` here subclasses
`torch.optim.Adam`, so construction, `param_groups`, `state_dict()` /
`load_state_dict()` and the per-parameter state (`step`, `exp_avg`,
`exp_avg_sq`) are torch's own and checkpoints move freely between the two;
only `step()` is replaced by `jabd_adam_step_f32` (csrc/adam.hip), which
applies torch's Adam arithmetic to all tensors of a group in a single
launch instead of torch's multi-kernel foreach chain.

Supported: fp32 CUDA tensors with contiguous params and dense grads, float
`lr`/`betas`, amsgrad / maximize / capturable / differentiable / fused /
decoupled_weight_decay all off (the reference's configuration).  Anything
else raises -- there is no silent fallback to torch's step.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .functional import _stream

_ROW_FIELDS = 5  # param, grad, exp_avg, exp_avg_sq, numel (struct AdamRow)


class Adam(torch.optim.Adam):
    """`torch.optim.Adam` with a single fused HIP step per parameter group."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                         amsgrad=amsgrad, **kw)
        self._tables = {}

    @staticmethod
    def _check_group(group):
        for key in ("amsgrad", "maximize", "capturable", "differentiable", "fused",
                    "decoupled_weight_decay"):
            if group.get(key):
                raise NotImplementedError(f"jabd_amd.optim.Adam: {key}=True is not supported")
        for key in ("lr", "eps", "weight_decay"):
            if isinstance(group[key], torch.Tensor):
                raise NotImplementedError(f"jabd_amd.optim.Adam: tensor {key} not supported")
        if any(isinstance(b, torch.Tensor) for b in group["betas"]):
            raise NotImplementedError("jabd_amd.optim.Adam: tensor betas not supported")

    def _table(self, tensors):
        """Device row + chunk tables for one launch, cached by the pointers."""
        key = tuple((p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel())
                    for p, g, m, v in tensors)
        hit = self._tables.get(key)
        if hit is not None:
            return hit
        dev = tensors[0][0].device
        rows = np.asarray(key, dtype=np.int64).reshape(-1, _ROW_FIELDS)
        numel = np.ascontiguousarray(rows[:, 4])
        nchunks = _lib.lib().jabd_adam_num_chunks(numel.ctypes.data, len(numel))
        chunks = np.empty(max(nchunks, 1), dtype=np.int64)
        _lib.call("jabd_adam_fill_chunks", numel.ctypes.data, len(numel), chunks.ctypes.data)
        hit = (torch.from_numpy(rows.copy()).to(dev), torch.from_numpy(chunks).to(dev), nchunks)
        if len(self._tables) > 64:
            self._tables.clear()
        self._tables[key] = hit
        return hit

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            self._check_group(group)
            beta1, beta2 = group["betas"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("jabd_amd.optim.Adam does not support sparse gradients")
                if (p.dtype != torch.float32 or g.dtype != torch.float32 or not p.is_cuda
                        or not p.is_contiguous() or not g.is_contiguous()):
                    raise NotImplementedError(
                        "jabd_amd.optim.Adam needs contiguous fp32 CUDA params and grads")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state["step"] += 1
                by_step.setdefault(float(state["step"]), []).append(
                    (p, g, state["exp_avg"], state["exp_avg_sq"]))
            for step, tensors in by_step.items():
                rows, chunks, nchunks = self._table(tensors)
                _lib.call("jabd_adam_step_f32", ctypes.c_void_p(rows.data_ptr()),
                          ctypes.c_void_p(chunks.data_ptr()), nchunks, float(group["lr"]),
                          float(beta1), float(beta2), float(group["eps"]),
                          float(group["weight_decay"]), 1.0 - beta1 ** step,
                          1.0 - beta2 ** step, _stream())
                # the kernel wrote through raw pointers: bump the version
                # counters as an in-place torch op would, so weight caches
                # keyed on _version (train._packed) see the new values
                torch.autograd.graph.increment_version([t[0] for t in tensors])
                # the training convs' packed weight copies, rebuilt in place
                # by one launch (instead of one per weight at the next forward)
                from . import train as _train
                _train.repack([t[0] for t in tensors])
        return loss
