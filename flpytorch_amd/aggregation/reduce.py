"""Server-side N-way reduction on MI355X — the ``serverGradient`` protocol.

Reference: every compressed-gradient algorithm folds the client models the same way,
``gs = w0 (x - x0); gs += wi (x - xi); gs / sum(w)`` in Buffer order
(fl_pytorch/utils/algorithms.py: DCGD 1748-1770, FedAvg 1810-1832, FedProx 1886-1908,
EF21 1521-1546, ...), then some return ``gs`` and the others pass it through the master
compressor (identity).  Here the fold is one ``flc_reduce_rows`` launch over a device array of
the client-model pointers — no stacking copy — bit-identical to the sequential torch loop.

Protocol kept from the reference (algorithms.py:2094-2125 and the class methods):
  * ``waitForItem()`` once per client before ``get(i)``; reads ``r['model']`` and
    ``r['client_state']['weight']``;
  * honours ``H['fl_dtype']`` and ``params_current.device`` (host tensors are moved to the GPU
    and the result moved back: the simulator's end-to-end path);
  * returns a new tensor the caller owns; 0 clients -> zeros.
"""
import ctypes

import torch

from .. import _lib


def _weights_and_total(weights):
    """Python-float weights as the reference uses them: each wi applied as fp32, the total summed
    as a python float in Buffer order and applied as the fp32 divisor."""
    total = weights[0]
    for w in weights[1:]:
        total += w
    uniform = all(float(w) == 1.0 for w in weights)
    return uniform, float(total)


def _work_device(t):
    """The GPU a tensor's fold runs on: its own device, or the current one for a host tensor."""
    _lib.require_gpu()
    return t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())


def reduce_rows(x, rows, weights=None, relative=True, out=None, divisor=None):
    """out = (sum_i w_i * (x - rows_i)) / sum(w)   (relative=True, client models in)
       out = (sum_i w_i * rows_i) / sum(w)         (relative=False, client updates in)

    ``rows`` is a list of fp32 device tensors shaped like ``x`` (or a 2-D [N, D] tensor), on
    ``x``'s device; ``x`` must be a device tensor (the callers move host tensors first).
    ``divisor`` replaces the fp32 divisor sum(w) (the multi-GPU block fold divides the sum of the
    block partials by the global client weight).
    """
    _lib.require_gpu()
    lib = _lib.load()
    if not x.is_cuda:
        raise ValueError("reduce_rows: x must be a device tensor (no CPU path)")
    dev = x.device
    n = rows.shape[0] if torch.is_tensor(rows) else len(rows)
    d = x.numel()
    if out is None:
        out = torch.empty_like(x)
    if n == 0:
        return out.zero_()
    weights = [1.0] * n if weights is None else [float(w) for w in weights]
    uniform, total = _weights_and_total(weights)
    if divisor is not None:
        total = float(divisor)
    keep = []
    w_ptr = None
    if not uniform:
        wt = torch.tensor(weights, dtype=torch.float32, device=dev)
        keep.append(wt)
        w_ptr = wt.data_ptr()
    x_ptr = x.data_ptr() if relative else None
    mode = _lib.FLC_REDUCE_REL_X if relative else _lib.FLC_REDUCE_PLAIN
    with torch.cuda.device(dev):
        if torch.is_tensor(rows) and rows.dim() == 2:
            rc = lib.flc_reduce_matrix(ctypes.c_void_p(rows.data_ptr()), rows.stride(0), n, d,
                                       ctypes.c_void_p(x_ptr), ctypes.c_void_p(w_ptr), ctypes.c_float(total), mode,
                                       ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(dev))
        else:
            rows = [r if (r.data_ptr() % 16 == 0 and r.is_contiguous()) else r.contiguous().clone() for r in rows]
            ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
            keep.append(ptrs)
            rc = lib.flc_reduce_rows(ctypes.c_void_p(ptrs.data_ptr()), n, d, ctypes.c_void_p(x_ptr),
                                     ctypes.c_void_p(w_ptr), ctypes.c_float(total), mode,
                                     ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(dev))
    _lib.check(rc, "flc_reduce")
    return out


def reduce_client_models(clients_responses, clients, params_current, H):
    """The shared core of the reference's serverGradient bodies (algorithms.py:1753-1768)."""
    if clients == 0:
        return torch.zeros_like(params_current)                  # algorithms.py:2117-2118
    fl_dtype = H["fl_dtype"]
    if fl_dtype != torch.float32 or params_current.dtype != torch.float32:
        raise TypeError(f"flcodec reduces fp32 only (fl_dtype={fl_dtype})")
    host = not params_current.is_cuda
    dev = _work_device(params_current)
    models, weights = [], []
    for i in range(clients):
        clients_responses.waitForItem()
        r = clients_responses.get(i)
        models.append(r["model"].to(device=dev, dtype=fl_dtype).reshape(-1))
        weights.append(r["client_state"]["weight"])
    x = params_current.to(device=dev).reshape(-1).contiguous()
    gs = reduce_rows(x, models, weights, relative=True)
    gs = gs.reshape(params_current.shape)
    return gs.to(params_current.device) if host else gs


def make_server_gradient(master_compress):
    """A ``serverGradient`` static method body: plain (FedAvg, FedProx) or followed by
    ``H['compressor_master'].compressVector`` (DCGD, EF21)."""

    def serverGradient(clients_responses, clients, model, params_current, H):
        gs = reduce_client_models(clients_responses, clients, params_current, H)
        if master_compress:
            return H["compressor_master"].compressVector(gs)
        return gs

    serverGradient.__doc__ = ("serverGradient on MI355X (flcodec reduce)" +
                              (" + master compressor" if master_compress else ""))
    return serverGradient


serverGradientPlain = make_server_gradient(False)
serverGradientMaster = make_server_gradient(True)


def serverGradientDIANA(clients_responses, clients, model, params_current, H):
    """DIANA.serverGradient (algorithms.py:1395-1421): the fold gs, recorded as H['m'] (the
    estimator without shift), returned shifted: H['h'] + gs."""
    gs = reduce_client_models(clients_responses, clients, params_current, H)
    H['m'] = gs
    return H['h'] + gs


def serverGradientGradSkip(clients_responses, clients, model, params_current, H):
    """GradSkip.serverGradient (algorithms.py:951-998): per client the bookkeeping of the
    reference (local_steps, shift refresh), the fold of x - (x_i - h_i * gamma / p) on MI355X,
    then delta_x = (x - gs) - x_i per client."""
    if clients == 0:
        return torch.zeros_like(params_current)
    for i in range(clients):
        clients_responses.waitForItem()
        cs = clients_responses.get(i)['client_state']
        cs['local_steps'].append(cs['Ki'])
        if cs['change_shift']:
            cs['hi'] = cs['grad']
            cs['stats']['send_scalars_to_master'] += 1
            cs['local_steps'][-1] += 1
    gamma = H['args'].local_lr
    fl_dtype = H["fl_dtype"]
    dev = params_current.device
    rows, weights = [], []
    for i in range(clients):
        cm = clients_responses.get(i)
        m = cm["model"].to(device=dev, dtype=fl_dtype) - cm['client_state']['hi'] * gamma / H['p']
        rows.append(m)
        weights.append(cm['client_state']['weight'])
    view = _ResponseView(rows, weights)
    gs = reduce_client_models(view, clients, params_current, H)
    x_mean = params_current - gs
    for i in range(clients):
        cm = clients_responses.get(i)
        cm['client_state']['delta_x'] = x_mean - cm["model"].to(device=dev, dtype=fl_dtype)
    return gs


def make_server_gradient_frecon(algorithms_module):
    """FRECON.serverGradient (algorithms.py:1124-1176): the model fold u and the fold of the
    clients' q_i (both on MI355X, client order), then
    q_avg + (1 - lambda) g_server_prev + lambda (u + h_prev) with lambda from the experiment options
    through the reference module's own helpers."""
    am = algorithms_module

    def serverGradient(clients_responses, clients, model, params_current, H):
        if clients == 0:
            return torch.zeros_like(params_current)
        u = reduce_client_models(clients_responses, clients, params_current, H)
        first = clients_responses.get(0)
        alpha = first["client_state"]['alpha']
        # the q fold runs on the GPU the model fold used (a host params_current: the current
        # device), its result returned to params_current's device
        dev = _work_device(params_current)
        qs, weights = [], []
        for i in range(clients):
            cs = clients_responses.get(i)['client_state']
            qs.append(cs['qi'].to(device=dev, dtype=H["fl_dtype"]).reshape(-1))
            weights.append(cs['weight'])
        ud = u.reshape(-1).to(dev)                                                       # x: shape only
        q_avg = reduce_rows(ud, qs, weights, relative=False).reshape(u.shape).to(params_current.device)
        for i in range(clients):
            del clients_responses.get(i)['client_state']['qi']
        h_prev = H['h_prev']
        if am.has_experiment_option(H, "lambda_"):
            lambda_ = am.get_experiment_option_f(H, "lambda_")
        elif am.has_experiment_option(H, "th_stepsize_noncvx") or am.has_experiment_option(H, "th_stepsize_cvx"):
            S = clients
            w = am.compressors.initCompressor(H["client_compressor"], H["D"]).getW()
            n = H['total_clients']
            H["lambda_th"] = S / (2 * (1 + w) * n)
            lambda_ = S / (2 * (1 + w) * n)
            am.get_logger(H).info(f"Used lambda is {lambda_}")
        else:
            raise UnboundLocalError("local variable 'lambda_' referenced before assignment")   # as the reference
        result = q_avg + (1.0 - lambda_) * H["g_server_prev"] + lambda_ * (u + h_prev)
        H['u_avg_update'] = u
        H['alpha_update'] = alpha * (clients / H['total_clients'])
        return result

    serverGradient.__doc__ = make_server_gradient_frecon.__doc__
    return serverGradient


class _ResponseView:
    """A Buffer-shaped view over precomputed client vectors (already waited for)."""

    def __init__(self, rows, weights):
        self.rows, self.weights = rows, weights

    def waitForItem(self):
        pass

    def get(self, i):
        return {"model": self.rows[i], "client_state": {"weight": self.weights[i]}}


def serverGradientCOFIG(clients_responses, clients, model, params_current, H):
    """COFIG.serverGradient (algorithms.py:1273-1307): the fold u = gs, returned as u + H['h_prev'];
    H['u_avg_update'] = u and H['alpha_update'] = alpha * (clients / H['total_clients']) with alpha
    the first response's client_state['alpha'] (for serverGlobalStateUpdate)."""
    if clients == 0:
        return torch.zeros_like(params_current)
    gs = reduce_client_models(clients_responses, clients, params_current, H)
    alpha = clients_responses.get(0)["client_state"]['alpha']
    result = gs + H['h_prev']
    H['u_avg_update'] = gs
    H['alpha_update'] = alpha * (clients / H['total_clients'])
    return result
