"""Flat parameter arena (flpytorch_amd/arena.py) against the flatten / unflatten semantics of
fl_pytorch/models/mutils.py:218-381 (restated below as the checker): same vectors bit for bit,
autograd writing into the arena, re-homing after set_to_none, training identical to a plain model."""
import copy
import types

import pytest
import torch

from flpytorch_amd import arena as ar


# -- checker: mutils' order and selection, one torch.cat / one slice assignment per tensor ----
def ref_params(model, skip=True):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters() if not (skip and not p.requires_grad)])


def ref_grads(model, skip=True):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                      for p in model.parameters() if not (skip and not p.requires_grad)])


def make_model(seed=0, freeze_first=True):
    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(3, 20, bias=False), torch.nn.Linear(20, 22), torch.nn.Tanh(),
                            torch.nn.Linear(22, 1))
    if freeze_first:
        m[0].requires_grad_(False)
    return m


def loss_of(m, x):
    return ((10.0 - m(x)) ** 2).mean()


@pytest.mark.parametrize("skip", [True, False])
def test_arena_vectors_match_mutils(skip):
    m = make_model()
    want_p = ref_params(m, skip)
    a = ar.FlatArena(m, skipFrozen=skip)
    assert a.D == want_p.numel()
    assert torch.equal(a.get_params(), want_p)
    x = torch.randn(5, 3)
    loss_of(m, x).backward()
    assert torch.equal(a.get_gradient(), ref_grads(m, skip))
    assert a.grad_view().data_ptr() == a.gflat.data_ptr()
    # set / add through the arena == what the parameters and grads then hold
    newp = torch.randn(a.D)
    a.set_params(newp)
    assert torch.equal(ref_params(m, skip), newp)
    g = torch.randn(a.D)
    a.set_gradient(g)
    assert torch.equal(ref_grads(m, skip), g)
    a.add_to_gradient(torch.ones(a.D))
    assert torch.equal(ref_grads(m, skip), g + torch.ones(a.D))
    assert torch.equal(a.get_zero_gradient_compatible_with_model(), torch.zeros(a.D))


def test_arena_survives_set_to_none_and_trains_identically():
    m1 = make_model(1)
    m2 = copy.deepcopy(m1)
    a = ar.FlatArena(m2)
    o1 = torch.optim.SGD([p for p in m1.parameters() if p.requires_grad], lr=0.05, momentum=0.9)
    o2 = torch.optim.SGD([p for p in m2.parameters() if p.requires_grad], lr=0.05, momentum=0.9)
    g = torch.Generator().manual_seed(3)
    for step in range(6):
        x = torch.randn(8, 3, generator=g)
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad(set_to_none=(step % 2 == 0))
            loss_of(m, x).backward()
            o.step()
        assert torch.equal(a.get_gradient(), ref_grads(m1))
        assert torch.equal(a.get_params(), ref_params(m1))
    # the views are the arena again after re-homing
    for p, off in zip(a.params, a.offsets):
        assert p.grad.data_ptr() == a.gflat[off:].data_ptr()
        assert p.data_ptr() == a.flat[off:].data_ptr()


def test_arena_install_and_fallback():
    calls = []

    def mk(name):
        def f(*args, **kw):
            calls.append(name)
            return name
        return f
    mod = types.SimpleNamespace(**{n: mk(n) for n in ("get_params", "set_params", "get_gradient", "set_gradient",
                                                      "add_to_gradient", "get_zero_gradient_compatible_with_model")})
    restore = ar.install(mod)
    m = make_model(2)
    plain = make_model(2)
    ar.FlatArena(m)
    assert torch.equal(mod.get_params(m), ref_params(m))
    assert calls == []
    assert mod.get_params(plain) == "get_params"                       # no arena: the reference code
    assert mod.get_params(m, True, lambda i, p: True) == "get_params"  # predicate: the reference code
    assert mod.get_gradient(m, skipFrozen=False) == "get_gradient"      # other selection: the reference
    restore()
    assert mod.get_params(m) == "get_params"


def test_arena_rejects_mixed_dtypes():
    m = make_model()
    m[1].double()
    with pytest.raises(TypeError):
        ar.FlatArena(m)
