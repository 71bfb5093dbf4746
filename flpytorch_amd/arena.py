"""Flat parameter arena: a model's trainable parameters and their gradients
re-homed as views into two flat [D] buffers, so the flatten / unflatten around the uplink kernels
(fl_pytorch/models/mutils.py:218-381: ``get_params`` / ``set_params`` / ``get_gradient`` /
``set_gradient`` / ``add_to_gradient`` / ``get_zero_gradient_compatible_with_model``, one
``torch.cat`` or one slice assignment per parameter tensor) becomes one contiguous copy — or no
copy at all through ``params_view()`` / ``grad_view()``, which the codec and reduction kernels
read in place.

Same order and selection as mutils (``model.parameters()`` order, frozen parameters skipped when
``skipFrozen``), same values bit for bit (copies only).  Gradients: autograd accumulates into an
existing ``.grad`` in place, so backward writes straight into the arena; when something replaces
a ``.grad`` (``zero_grad(set_to_none=True)``, the default, sets it to None) the arena re-homes it
on the next gradient access.  ``param_predicate`` subsets are not an arena shape: the module-level
wrappers installed by ``install()`` fall back to the reference functions for them.
"""
import torch


class FlatArena:
    def __init__(self, model: torch.nn.Module, skipFrozen: bool = True):
        self.model = model
        self.skipFrozen = skipFrozen
        self.params = [p for p in model.parameters() if not (skipFrozen and not p.requires_grad)]
        if not self.params:
            raise ValueError("FlatArena: the model has no parameters to hold")
        dtypes = {p.dtype for p in self.params}
        devices = {p.device for p in self.params}
        if len(dtypes) != 1 or len(devices) != 1:
            raise TypeError("FlatArena: parameters must share one dtype and one device")
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += p.numel()
        self.D = off
        dev, dt = next(iter(devices)), next(iter(dtypes))
        self.flat = torch.empty(self.D, dtype=dt, device=dev)
        self.gflat = torch.zeros(self.D, dtype=dt, device=dev)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p.numel()
                self.flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + n].view_as(p)
                if p.grad is not None:
                    self.gflat[o:o + n].copy_(p.grad.reshape(-1))
                p.grad = self.gflat[o:o + n].view_as(p)
        model._flc_arena = self

    # -- zero-copy access -------------------------------------------------------------------
    def params_view(self):
        return self.flat

    def grad_view(self):
        self._rehome_grads()
        return self.gflat

    def _rehome_grads(self):
        """Put every parameter's .grad back into the arena (after a set_to_none / replacement);
        a missing gradient reads as zeros, like mutils.get_gradient."""
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p.numel()
                view = self.gflat[o:o + n]
                g = p.grad
                if g is not None and g.data_ptr() == view.data_ptr() and g.is_contiguous():
                    continue
                if g is None:
                    view.zero_()
                else:
                    view.copy_(g.reshape(-1))
                p.grad = view.view_as(p)
        # parameters whose .data was rebound elsewhere (load_state_dict keeps storage; a user
        # assigning p.data would not) are brought back too
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p.numel()
                if p.data.data_ptr() != self.flat[o:o + n].data_ptr():
                    self.flat[o:o + n].copy_(p.data.reshape(-1))
                    p.data = self.flat[o:o + n].view_as(p)

    # -- mutils.py:218-381 shapes, one copy each ---------------------------------------------
    def get_params(self):
        self._rehome_grads()
        return self.flat.clone()

    def set_params(self, parameters):
        self._rehome_grads()
        with torch.no_grad():
            self.flat.copy_(parameters.reshape(-1)[:self.D])

    def get_gradient(self):
        return self.grad_view().clone()

    def set_gradient(self, grad):
        self._rehome_grads()
        with torch.no_grad():
            self.gflat.copy_(grad.reshape(-1)[:self.D])

    def add_to_gradient(self, extra_grad):
        self._rehome_grads()
        with torch.no_grad():
            self.gflat.add_(extra_grad.reshape(-1)[:self.D])

    def get_zero_gradient_compatible_with_model(self):
        return torch.zeros_like(self.gflat)


def _arena_for(model, skipFrozen, param_predicate):
    a = getattr(model, "_flc_arena", None)
    if a is None or param_predicate is not None or a.skipFrozen != skipFrozen:
        return None
    return a


def install(mutils_module):
    """Rebind mutils' flatten / unflatten functions to use a model's arena when it has one
    (``FlatArena(model)``), the reference code otherwise.  Returns a restore callable."""
    saved = {name: getattr(mutils_module, name) for name in
             ("get_params", "set_params", "get_gradient", "set_gradient", "add_to_gradient",
              "get_zero_gradient_compatible_with_model")}

    def get_params(model, skipFrozen=True, param_predicate=None):
        a = _arena_for(model, skipFrozen, param_predicate)
        return a.get_params() if a else saved["get_params"](model, skipFrozen, param_predicate)

    def set_params(model, parameters, skipFrozen=True, param_predicate=None):
        a = _arena_for(model, skipFrozen, param_predicate)
        return a.set_params(parameters) if a else saved["set_params"](model, parameters, skipFrozen, param_predicate)

    def get_gradient(model, skipFrozen=True):
        a = _arena_for(model, skipFrozen, None)
        return a.get_gradient() if a else saved["get_gradient"](model, skipFrozen)

    def set_gradient(model, grad, skipFrozen=True):
        a = _arena_for(model, skipFrozen, None)
        return a.set_gradient(grad) if a else saved["set_gradient"](model, grad, skipFrozen)

    def add_to_gradient(model, extra_grad, skipFrozen=True):
        a = _arena_for(model, skipFrozen, None)
        return a.add_to_gradient(extra_grad) if a else saved["add_to_gradient"](model, extra_grad, skipFrozen)

    def get_zero_gradient_compatible_with_model(model, skipFrozen=True):
        a = _arena_for(model, skipFrozen, None)
        return a.get_zero_gradient_compatible_with_model() if a else \
            saved["get_zero_gradient_compatible_with_model"](model, skipFrozen)

    for name, fn in [("get_params", get_params), ("set_params", set_params), ("get_gradient", get_gradient),
                     ("set_gradient", set_gradient), ("add_to_gradient", add_to_gradient),
                     ("get_zero_gradient_compatible_with_model", get_zero_gradient_compatible_with_model)]:
        setattr(mutils_module, name, fn)

    def restore():
        for name, fn in saved.items():
            setattr(mutils_module, name, fn)
    return restore
