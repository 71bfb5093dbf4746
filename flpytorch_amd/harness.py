"""The simulated communication round of FL_PyTorch, driven through the MI355X uplink.

The reference's round restated around the product: the host orchestration stays
Python like the reference's, every codec call and the server fold run in libflcodec.so.

  run.py:343-369          np_random.seed(manual_runtime_seed); all rounds' clients pre-sampled
                          (fl_funcs.py:12-43: uniform = choice(n, m, replace=False) per round;
                          poisson = one uniform() per client per round)
  model_funcs.py:459-614  run_one_communication_round: per sampled client, in order,
                          algorithms.clientState (DCGD 1729-1732: initCompressor +
                          generateCompressPattern on the shared stream; then every algorithm's
                          seed draw randint(2**31), algorithms.py:2055) and local_training;
                          then the aggregation block: serverGradient, global optimiser step,
                          serverGlobalStateUpdate
  model_funcs.py:617-723  train_model: per local iteration f, g = local gradient at x_i
                          (algorithms.py:24-113 evaluateGradient, internal_sgd:full-gradient),
                          c = C(g) (DCGD 1735-1745) or g (FedAvg 1797-1807), x_i -= lr * c (SGD,
                          momentum 0: torch.optim.SGD's param.add_(grad, alpha=-lr))
  algorithms.py:2153-2223 serverGlobalStateUpdate: history[round] = {grad_sgd_server_l2 = ||gs||,
                          x_before_round = ||x||, approximate_f_avg_value = mean of the clients'
                          f values, client_states}; l2 = sqrt(sum(v**2).item()) (mutils.py:395)

Where the work runs: the codecs (``Compressor.compressVector``, compat patterns from the shared
numpy stream) and the fold (``serverGradient`` -> flc_reduce_rows) on the GPU, always; the
model-side local gradient (out of the hot path) on the device of the iterate:
``device="cpu"`` mirrors the reference's ``--gpu -1`` runs (config C1: client rows cross to the
GPU for the codec and the fold and back), ``device="cuda"`` keeps the whole round on the MI355X.

Algorithms driven here: DCGD (client step ``C(g)``), FedAvg (``g``), and the shifted ones whose
client step is the fused shift codec (``Compressor.compressShift``, one flc_encode_shift pass):

  DIANA   algorithms.py:1317-1428  h0 = h = 0 or the full gradient at x0 (get_initial_shift,
                                   474-479; run.py:408-418), alpha = 1 / (1 + w); client i keeps
                                   h_i across rounds (findRecentRecordAndRemoveFromHistory,
                                   371-399); step m_i = C(g - h_i), h_i += alpha m_i (dianaStep);
                                   server: gs = fold, H['m'] = gs, returns h + gs, then
                                   h += alpha m
  EF21    algorithms.py:1432-1554  round 0 samples every client (request_use_full_list_of_clients,
                                   model_funcs.py:470-475); a client's first step sends g and keeps
                                   it as g_i; later g_i += C(g - g_i) * mult (ef21Step, mult =
                                   1 / (1 + w) unless C is a contraction); server: fold + master
                                   (identity) compressor

The others' serverGradient bodies are covered by ``aggregation.install``.
"""
import math
import threading

import numpy as np
import torch
import torch.nn.functional as F

from . import aggregation as ag
from . import transport


# ---------------------------------------------------------------------------------------------
# client sampling (fl_funcs.py:12-43)
# ---------------------------------------------------------------------------------------------
def get_sampled_clients(num_clients, clients_per_round, rounds, np_random, sampling="uniform", poisson_p=None):
    """All rounds' sampled clients, drawn up front from the experiment stream like the reference."""
    if sampling == "uniform":
        return [np_random.choice(num_clients, clients_per_round, replace=False) for _ in range(rounds)]
    if sampling in ("poisson", "poisson-no-empty"):
        out = []
        for _ in range(rounds):
            picked = []
            while True:
                for j in range(num_clients):
                    if np_random.uniform() < poisson_p:
                        picked.append(j)
                if picked or sampling == "poisson":
                    break
            out.append(np.asarray(picked))
        return out
    raise AssertionError("Unknown sampling type!")                         # fl_funcs.py:42


# ---------------------------------------------------------------------------------------------
# the model side: local objective of one client
# ---------------------------------------------------------------------------------------------
class DenseModel:
    """model "dense" (model_funcs.py:170-189): Flatten, Linear(d, 32), ReLU, Linear(32, 64), ReLU,
    Linear(64, out), Sigmoid, on a flat parameter vector laid out as ``model.parameters()`` is
    (mutils.get_params, mutils.py:218-255: W1, b1, W2, b2, W3, b3).  Loss: MSELoss(reduction='sum')
    (model_funcs.py:133) scaled by 1 / n_samples per batch (algorithms.py:89-90), full gradient
    over the client's data in batches of ``batch_size`` (the DataLoader, shuffle=False)."""

    def __init__(self, data, targets, samples_per_client, batch_size=32):
        self.data = torch.as_tensor(data, dtype=torch.float32)
        self.targets = torch.as_tensor(targets, dtype=torch.float32)
        self.spc = int(samples_per_client)
        self.batch_size = int(batch_size)
        d_in, d_out = self.data[0].numel(), self.targets[0].numel()
        self.shapes = [(32, d_in), (32,), (64, 32), (64,), (d_out, 64), (d_out,)]
        self.D = sum(math.prod(s) for s in self.shapes)
        self._dev = {}

    def _client_data(self, client, device):
        key = (str(device), None if client is None else int(client))
        if key not in self._dev:
            if client is None:                                  # set_client(None): the whole train set
                self._dev[key] = (self.data.to(device), self.targets.to(device))  # (artificial_dataset.py:156-158)
            else:
                lo = int(client) * self.spc
                self._dev[key] = (self.data[lo:lo + self.spc].to(device),
                                  self.targets[lo:lo + self.spc].to(device))
        return self._dev[key]

    def value_and_gradient(self, x, client):
        """(f, g): the client's loss at x as a Python float (evaluateGradient's
        function_value.item(), algorithms.py:112) and its gradient as a flat [D] fp32 tensor on
        x's device (mutils.get_gradient).  ``client=None``: the whole train set (run.py:408-413)."""
        params, off = [], 0
        for s in self.shapes:
            n = math.prod(s)
            params.append(x[off:off + n].detach().view(s).clone().requires_grad_(True))
            off += n
        data, targets = self._client_data(client, x.device)
        total = data.shape[0]
        fval = torch.zeros(1, dtype=torch.float32, device=x.device)
        grads = None
        for b0 in range(0, total, self.batch_size):
            xb = data[b0:b0 + self.batch_size].flatten(1)
            yb = targets[b0:b0 + self.batch_size]
            h = F.relu(F.linear(xb, params[0], params[1]))
            h = F.relu(F.linear(h, params[2], params[3]))
            out = torch.sigmoid(F.linear(h, params[4], params[5]))
            loss = F.mse_loss(out, yb, reduction="sum") * (1.0 / total)
            fval = fval + loss.detach()
            gb = torch.autograd.grad(loss, params)
            grads = list(gb) if grads is None else [a + b for a, b in zip(grads, gb)]   # .grad accumulation
        g = torch.cat([t.reshape(-1) for t in grads])
        return fval.item(), g


# ---------------------------------------------------------------------------------------------
# the round
# ---------------------------------------------------------------------------------------------
def l2_norm_of_vec(v):
    """mutils.l2_norm_of_vec (mutils.py:395-396): sqrt of the fp32 sum of squares, as a float."""
    return ((v ** 2).sum().item()) ** 0.5


class _Buffer:
    """The reference's Buffer contract as serverGradient consumes it (buffer.py:7-105): items in
    push order, one waitForItem() per get()."""

    def __init__(self):
        self.items = []

    def pushBack(self, item):
        self.items.append(item)

    def waitForItem(self):
        pass

    def get(self, i):
        return self.items[i]

    def __len__(self):
        return len(self.items)


def find_recent_and_remove(H, client_id, field):
    """findRecentRecordAndRemoveFromHistory (algorithms.py:371-399): the newest round that sampled
    the client holds the field (None after a previous read) or ends the search."""
    for r in sorted(H["history"], reverse=True):
        states = H["history"][r]["client_states"]
        if client_id in states:
            st = states[client_id]["client_state"]
            if field in st:
                v, st[field] = st[field], None
                return v
            return None
    return None


def _on_gpu(step):
    """Run a shift-codec client step on the MI355X whatever device the client state lives on
    (``device="cpu"``: the --gpu -1 layout, tensors cross to the GPU and back like the DCGD codec)."""
    def run(comp, *tensors, **kw):
        home = tensors[0].device
        if home.type == "cuda":
            return step(comp, *tensors, **kw)
        out = step(comp, *[t.cuda() if torch.is_tensor(t) else t for t in tensors], **kw)
        return tuple(o.to(home) for o in out) if isinstance(out, tuple) else out.to(home)
    return run


ALGORITHMS = ("dcgd", "fedavg", "diana", "ef21", "marina")


class Simulation:
    """One experiment: ``rounds`` communication rounds of ``algorithm`` (one of ``ALGORITHMS``)
    with the client codec ``client_compressor`` (the reference's spec grammar), starting at ``x0``.

    ``init_compressor`` / ``server_gradient`` / ``diana_step`` / ``ef21_step`` / ``marina_step``
    default to the product (flpytorch_amd.aggregation: HIP codecs, HIP fold, fused shift codec);
    tests may pass other implementations of the same protocol."""

    def __init__(self, algorithm, client_compressor, model, x0, num_clients, clients_per_round, rounds,
                 local_lr, global_lr, local_iters=1, runtime_seed=0, device="cuda", sampling="uniform",
                 poisson_p=None, init_compressor=None, server_gradient=None, record_iterates=False, wire=False,
                 initialize_shifts_policy="zero", diana_step=None, ef21_step=None, marina_step=None):
        algorithm = algorithm.lower()
        if algorithm not in ALGORITHMS:
            raise ValueError(f"harness drives {', '.join(ALGORITHMS)}, not {algorithm!r}")  # algorithms.py:1954 style
        if wire and algorithm != "dcgd":
            raise ValueError("wire mode drives DCGD's compressVector messages only")
        if initialize_shifts_policy not in ("zero", "full_gradient_at_start"):
            raise ValueError(f"unknown initialize_shifts_policy {initialize_shifts_policy!r}")  # opts.py:437-441
        self.algorithm = algorithm
        self.spec = client_compressor.lower()                                    # opts.py:497 lowercases argv
        self.model = model
        self.device = torch.device(device)
        self.x = torch.as_tensor(x0, dtype=torch.float32).reshape(-1).to(self.device).clone()
        self.D = self.x.numel()
        self.num_clients, self.per_round, self.rounds = int(num_clients), int(clients_per_round), int(rounds)
        self.local_lr, self.global_lr, self.local_iters = float(local_lr), float(global_lr), int(local_iters)
        self.record_iterates = record_iterates
        # wire=True (DCGD): each client's compressed gradient crosses the "network" as the wire
        # message (Compressor.compressPayload, include/flcodec.h layouts) and the server side
        # rebuilds it (decompressPayload, bit-exact) before the local step it applies — the
        # physical form of last_need_to_send_advance (the reference pickles dense tensors,
        # comm_socket.py:16-82); bytes per client in client_state["stats"]["payload_bytes"].
        # wire="socket": the message also crosses a real socket (transport.PayloadSocket,
        # CommSocket framing) and is checked against the codec on arrival (validatePayload)
        if wire not in (False, True, "socket"):
            raise ValueError(f"wire must be False, True or 'socket' (got {wire!r})")
        self.wire = wire
        self.link = transport.socket_pair() if wire == "socket" else None
        self.iterates = []                                                       # x after each round (opt-in)
        self.init_compressor = init_compressor or ag.initCompressor
        self.diana_step = diana_step or _on_gpu(ag.dianaStep)
        self.ef21_step = ef21_step or _on_gpu(ag.ef21Step)
        self.marina_step = marina_step or _on_gpu(ag.marinaStep)
        # DCGD / EF21 fold then apply the master (identity) compressor (algorithms.py:1748-1770,
        # 1521-1546); FedAvg and MARINA return the fold (1810-1832, 545-563); DIANA returns h + fold
        # (1395-1421)
        default_fold = {"dcgd": ag.serverGradientMaster, "ef21": ag.serverGradientMaster,
                        "fedavg": ag.serverGradientPlain, "diana": ag.serverGradientDIANA,
                        "marina": ag.serverGradientPlain}[algorithm]
        self.server_gradient = server_gradient or default_fold
        self.np_random = np.random.RandomState()
        self.np_random.seed(int(runtime_seed))                                   # run.py:343-345
        self.sampled = get_sampled_clients(self.num_clients, self.per_round, self.rounds, self.np_random,
                                           sampling, poisson_p)                  # run.py:369
        master = ag.Compressor()
        master.makeIdenticalCompressor()                                         # DCGD/initializeServerState
        self.H = {"algorithm": algorithm, "D": self.D, "fl_dtype": torch.float32, "client_compressor": self.spec,
                  "compressor_master": master, "total_clients": self.num_clients, "history": {}}
        if algorithm == "dcgd":
            c = self.init_compressor(self.spec, self.D)
            if c.isUnbiasedCompressor():
                self.H["w"] = c.getW()
            elif c.isContractionCompressor():
                self.H["alpha"] = c.getAlphaContraction()
        elif algorithm == "diana":                                               # algorithms.py:1346-1357
            w = self.init_compressor(self.spec, self.D).getW()
            if initialize_shifts_policy == "full_gradient_at_start":             # run.py:408-413
                _, h0 = self.model.value_and_gradient(self.x, None)
            else:
                h0 = torch.zeros(self.D, dtype=torch.float32, device=self.device)
            self.H.update({"h0": h0.detach().clone(), "h": h0.detach().clone(), "alpha": 1.0 / (1.0 + w), "w": w})
        elif algorithm == "ef21":                                                # algorithms.py:1460-1468
            self.H["request_use_full_list_of_clients"] = True
        elif algorithm == "marina":                                              # algorithms.py:486-492
            # test_ber_rv = 0 forces a full-gradient first round
            self.H.update({"x_prev": self.x.clone(), "test_ber_rv": 0.0})

    # algorithms.clientState (2015-2069) with the class parts: DCGD 1729-1732, FedAvg 1793-1794,
    # DIANA 1360-1373, EF21 1471-1484, MARINA 495-509
    def client_state(self, client_id, rnd):
        cs = {}
        if self.algorithm in ("dcgd", "diana", "ef21", "marina"):
            comp = self.init_compressor(self.H["client_compressor"], self.D)
            comp.generateCompressPattern(self.np_random, str(self.device), client_id, self.H)
            cs["client_compressor"] = comp
        if self.algorithm == "marina":
            p = 1.0 / (1.0 + comp.getW())
            cs.update({"p": p, "ck": 1 if self.H["test_ber_rv"] <= p else 0})
        if self.algorithm == "diana":
            hi = find_recent_and_remove(self.H, client_id, "hi")
            cs["hi"] = self.H["h0"].detach().clone() if hi is None else hi
        elif self.algorithm == "ef21":
            cs["g_prev"] = find_recent_and_remove(self.H, client_id, "g_prev")
        cs.update({"algorithm": self.algorithm, "client_id": client_id, "weight": 1.0, "round": rnd,
                   "approximate_f_value": [], "seed": self.np_random.randint(2 ** 31),
                   "stats": {"send_scalars_to_master": 0}})
        return cs

    # the class's localGradientEvaluation after the gradient is known: the vector the local SGD
    # step applies
    def client_step(self, cs, g):
        comp = cs.get("client_compressor")
        if self.algorithm == "fedavg":                                           # algorithms.py:1803-1807
            cs["stats"]["send_scalars_to_master"] += g.numel()
            return g
        if self.algorithm == "dcgd":                                             # algorithms.py:1741-1745
            if self.wire:
                msg = comp.compressPayload(g)
                cs["stats"]["payload_bytes"] = cs["stats"].get("payload_bytes", 0) + msg.numel()
                if self.link is not None:
                    msg = self.transfer(comp, msg, g.numel())
                c = comp.decompressPayload(msg, g.numel())
            else:
                c = comp.compressVector(g)
            cs["stats"]["send_scalars_to_master"] += comp.last_need_to_send_advance
            return c
        if self.algorithm == "diana":                                            # algorithms.py:1383-1392
            m, cs["hi"] = self.diana_step(comp, g, cs["hi"], self.H["alpha"])
            cs["stats"]["send_scalars_to_master"] += comp.last_need_to_send_advance
            return m
        if self.algorithm == "marina":                                           # algorithms.py:512-540
            if cs["ck"] == 1:
                cs["stats"]["send_scalars_to_master"] += g.numel()
                return g
            # the gradient at the previous iterate (its function value is not recorded), then
            # g_prev + C(grad_cur - grad_prev) in one fused pass
            _, g_old = self.model.value_and_gradient(self.H["x_prev"], cs["client_id"])
            g_next = self.marina_step(comp, g, g_old, self.H["g_prev"].to(g.device))
            cs["stats"]["send_scalars_to_master"] += comp.last_need_to_send_advance
            return g_next
        if cs["g_prev"] is None:                                                 # EF21, algorithms.py:1494-1500
            cs["g_prev"] = g                                                     # (first step: not counted)
            return g
        g_next = self.ef21_step(comp, g, cs["g_prev"])                           # algorithms.py:1502-1518
        cs["stats"]["send_scalars_to_master"] += comp.last_need_to_send_advance
        cs["g_prev"] = g_next
        return g_next

    def transfer(self, comp, msg, d):
        """One message client -> server over the socket pair: the client end sends on a thread
        (a message larger than the socket buffer would otherwise block), the server end receives
        and validates it; returns the received host uint8 tensor."""
        client, server = self.link
        err = []

        def send():
            try:
                client.sendPayload(msg)
            except Exception as e:                      # surfaced after the join
                err.append(e)
        t = threading.Thread(target=send, daemon=True)
        t.start()
        try:
            got = server.recvPayload(comp, d)
        except BaseException:
            # a refused or broken message: unblock the sender (it may sit in sendall on a full
            # socket buffer) before waiting for it
            server.abort()
            client.abort()
            t.join(timeout=30)
            raise
        t.join()
        if err:
            raise err[0]
        return got

    # local_training (model_funcs.py:318-388) + train_model's loop (617-723)
    def local_training(self, cs, client_id):
        xi = self.x.clone()
        for _ in range(self.local_iters):
            f, g = self.model.value_and_gradient(xi, client_id)
            c = self.client_step(cs, g)
            cs["approximate_f_value"].append(f)
            xi.add_(c.to(xi.device), alpha=-self.local_lr)                      # SGD step, momentum 0
        return {"model": xi, "client_id": client_id, "client_state": cs}

    # run_one_communication_round (model_funcs.py:459-614)
    def run_round(self, rnd):
        if self.H.get("request_use_full_list_of_clients"):                       # model_funcs.py:470-475
            clients = np.arange(self.H["total_clients"])
        else:
            clients = self.sampled[rnd]
        buf = _Buffer()
        for cid in clients:
            cs = self.client_state(int(cid), rnd)
            buf.pushBack(self.local_training(cs, int(cid)))
        n = len(clients)
        x_prev = self.x.clone()
        if n == 0:
            gs = torch.zeros_like(self.x)                                        # algorithms.py:2117-2118
        else:
            gs = self.server_gradient(buf, n, None, x_prev, self.H)
        self.x.add_(gs, alpha=-self.global_lr)                                   # global SGD step
        if self.record_iterates:
            self.iterates.append(self.x.detach().cpu().clone())
        fvalues = []
        states = {}
        for item in buf.items:
            fvalues += item["client_state"]["approximate_f_value"]
            st = item["client_state"]
            st.pop("client_compressor", None)                                    # algorithms.py:2198-2199
            states[item["client_id"]] = {"client_state": st}
        self.H["history"][rnd] = {
            "client_states": states,
            "grad_sgd_server_l2": l2_norm_of_vec(gs),
            "approximate_f_avg_value": float(np.mean(fvalues)) if fvalues else float("nan"),
            "x_before_round": l2_norm_of_vec(x_prev),
        }
        # the class's serverGlobalStateUpdate (2239-2240)
        if self.algorithm == "diana":                                            # algorithms.py:1424-1428
            self.H["h"] = self.H["h"] + self.H["alpha"] * self.H["m"]
        elif self.algorithm == "ef21":                                           # algorithms.py:1549-1554
            self.H["compressor_master"].generateCompressPattern(self.np_random, str(self.device), -1, self.H)
            self.H["request_use_full_list_of_clients"] = False
        elif self.algorithm == "marina":                                         # algorithms.py:566-572
            self.H["g_prev"] = gs
            self.H["x_prev"] = self.x.clone()                                    # the iterate after the step
            self.H["test_ber_rv"] = self.np_random.random()
        return self.H["history"][rnd]

    def run(self):
        for r in range(self.rounds):
            prev = self.H["history"].get(r - 1)
            if prev is not None and any(math.isnan(prev[k]) or math.isinf(prev[k])
                                        for k in ("x_before_round", "grad_sgd_server_l2")):
                break                                                            # run.py:466-479
            self.run_round(r)
        return self.H
