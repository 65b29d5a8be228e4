"""Base class of every nn.Module this package exports, and its pack caches.

Eval mode folds BatchNorm into the convolutions and packs the weights into
the MFMA fragment order once; the packed tensors live in a per-module cache
keyed by device (so nn.DataParallel replicas on GPU k, which share the
original's __dict__ shallowly, each get packs built from their own
broadcast parameters, once).  Staleness is tracked with one process-wide
generation counter that every event able to change a parameter bumps:

  * Module.train() / .eval()      (an optimizer step happens in train mode)
  * Module._apply()               (.to(), .cuda(), .float(), ...)
  * Module._load_from_state_dict  (load_state_dict at any depth)
  * invalidate()                  (explicit, after editing weights in place
                                   while the model stays in eval mode)

so a forward does O(1) host work to validate its packs (checking every
parameter's version would be O(params) per call, which a bs1 predict loop
feels).  An entry also records the storage address of the module's first
parameter: a module whose parameters are different tensors than the ones its
packs were built from (an nn.DataParallel replica holding freshly broadcast
weights, or weights swapped in with setattr/load) rebuilds them.  Training
mode never reads these caches.
"""
import threading

import torch
import torch.nn as nn

_GEN = [0]
_LOCK = threading.Lock()


def invalidate():
    """Drop every eval-mode pack (call after editing parameters in place in
    eval mode without going through train()/eval()/to()/load_state_dict())."""
    with _LOCK:
        _GEN[0] += 1


def generation():
    return _GEN[0]


def _first_param_ptr(module):
    """data_ptr of the first parameter under `module` (a replicate()d module
    keeps its broadcast parameters as plain attributes listed in
    _former_parameters, not in _parameters)."""
    for m in module.modules():
        for t in m._parameters.values():
            if t is not None:
                return t.data_ptr()
        for k in m.__dict__.get("_former_parameters", {}):
            t = m.__dict__.get(k)  # the attribute the forward reads
            if isinstance(t, torch.Tensor):
                return t.data_ptr()
    return 0


class HipModule(nn.Module):
    """Mixin placed before the torch base class: `class Conv2d(HipModule, nn.Conv2d)`.

    Adds the eval pack cache and its invalidation events; adds no
    parameters, buffers or state_dict keys."""

    def _jabd_cached(self, device, build, tag=None):
        cache = self.__dict__.get("_jabd_cache")
        if cache is None:
            cache = self.__dict__["_jabd_cache"] = {}
        key = (device.type, device.index, tag)
        gen = _GEN[0]
        probe = _first_param_ptr(self)
        ent = cache.get(key)
        if ent is None or ent[0] != gen or ent[1] != probe:
            with torch.no_grad():
                ent = (gen, probe, build())
            cache[key] = ent
        return ent[2]

    def train(self, mode=True):
        invalidate()
        return super().train(mode)

    def _apply(self, fn, recurse=True):
        invalidate()
        return super()._apply(fn, recurse)

    def _load_from_state_dict(self, *args, **kwargs):
        invalidate()
        return super()._load_from_state_dict(*args, **kwargs)

    def _replicate_for_data_parallel(self):
        # make sure the cache dict exists on the original so every replica
        # (a shallow __dict__ copy) shares it; entries are keyed by device
        self.__dict__.setdefault("_jabd_cache", {})
        return super()._replicate_for_data_parallel()
