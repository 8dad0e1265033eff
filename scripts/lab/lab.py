"""Algorithm lab (dev study): iteration counts of PDHG variants on config-4 windows, cold and seeded-warm, on host
cores via scripts/lab/liblab.so (a knob-carrying copy of oracle/cpu_pdhg.cpp).

Usage: python scripts/lab/lab.py <scenarios> <variant-json> [<variant-json> ...]
  a variant is a JSON object of LAB_* environment knobs and dvh_options fields, e.g.
  '{}' '{"LAB_KP": 0.99, "LAB_KI": 0.01}' '{"LAB_BOR": 1}' '{"primal_weight_theta": 0.5}'
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import numpy as np  # noqa: E402

from dervet_hip import _lib  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402
from dervet_hip.sweep import seed_split  # noqa: E402

LIB = os.path.join(HERE, "liblab.so")


class Lab:
    def __init__(self):
        self.lib = _lib.load(LIB)
        self.lib.lab_set_traj.argtypes = [ctypes.c_void_p]
        self.lib.lab_set_pw.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        self.opts = _lib.Options()
        self.lib.dvh_default_options(ctypes.byref(self.opts))
        h = ctypes.c_void_p()
        assert self.lib.dvh_create(1, ctypes.byref(self.opts), ctypes.byref(h)) == 0
        self.h = h

    def solve(self, lps, starts=None, pw_in=None, **opts):
        o = _lib.Options()
        ctypes.memmove(ctypes.byref(o), ctypes.byref(self.opts), ctypes.sizeof(o))
        for k, v in opts.items():
            setattr(o, k, v)
        self.lib.dvh_set_options(self.h, ctypes.byref(o))
        n = len(lps)
        arr, res = (_lib.LP * n)(), (_lib.Result * n)()
        keep, outs = [], []

        def ptr(a, t, ct):
            a = np.ascontiguousarray(a, dtype=t)
            keep.append(a)
            return a.ctypes.data_as(ct)
        for k, lp in enumerate(lps):
            a = arr[k]
            a.n, a.m_eq, a.m_ineq, a.nnz = lp.n, lp.m_eq, lp.m - lp.m_eq, len(lp.indices)
            a.indptr, a.indices = ptr(lp.indptr, np.int32, _lib.c_int32_p), ptr(lp.indices, np.int32, _lib.c_int32_p)
            a.data, a.c = ptr(lp.data, np.float64, _lib.c_double_p), ptr(lp.c, np.float64, _lib.c_double_p)
            a.q, a.l = ptr(lp.q, np.float64, _lib.c_double_p), ptr(lp.l, np.float64, _lib.c_double_p)
            a.u, a.c0 = ptr(lp.u, np.float64, _lib.c_double_p), lp.c0
            x, y = np.zeros(lp.n), np.zeros(lp.m)
            if starts is not None:
                x[:], y[:] = starts[k]
            outs.append((x, y))
            res[k].x = x.ctypes.data_as(_lib.c_double_p)
            res[k].y = y.ctypes.data_as(_lib.c_double_p)
        traj = np.full((n, 3), -1, np.int32)
        self.lib.lab_set_traj(traj.ctypes.data)
        pw_out, pw0_out = np.zeros(n), np.zeros(n)
        pin = None if pw_in is None else np.ascontiguousarray(pw_in, np.float64)
        self.lib.lab_set_pw(None if pin is None else pin.ctypes.data, pw_out.ctypes.data, pw0_out.ctypes.data)
        t = time.perf_counter()
        assert self.lib.dvh_solve_batch(self.h, arr, n, res) == 0
        wall = time.perf_counter() - t
        self.lib.lab_set_traj(None)
        self.lib.lab_set_pw(None, None, None)
        it = np.array([res[k].iters for k in range(n)])
        st = np.array([res[k].status for k in range(n)])
        obj = np.array([res[k].obj for k in range(n)])
        return dict(iters=it, status=st, obj=obj, x=[o[0] for o in outs], y=[o[1] for o in outs], traj=traj, wall=wall,
                    pw=pw_out, pw0=pw0_out)


def transfer(lp_r, lp_s, xs, ys):
    """sweep.transfer for one window pair (numpy)."""
    ok = np.isfinite(lp_r.u) & np.isfinite(lp_s.u) & (lp_s.u > 0)
    ratio = np.where(ok, lp_r.u / np.where(ok, lp_s.u, 1.0), 1.0)
    x = xs * ratio
    y = ys.copy()
    T = lp_r.m_eq - 1
    if lp_r.n == 3 * T + 1 and os.environ.get("LAB_TAU_SCALE"):  # the demand column by the ratio of peak net loads
        qr, qs = np.abs(lp_r.q[T + 1:]).max(), np.abs(lp_s.q[T + 1:]).max()
        if qs > 0:
            x[3 * T] = xs[3 * T] * qr / qs
    if lp_r.n == 3 * T + 1:
        cd = lp_r.c[3 * T] / max(lp_s.c[3 * T], 1e-12)
        cp = np.abs(lp_r.c[:T]).mean() / max(np.abs(lp_s.c[:T]).mean(), 1e-12)
        y[:T + 1] *= cp
        y[T + 1:] *= cd
    return x, y


def summary(tag, r, base_obj=None):
    it = r["iters"]
    tr = r["traj"]
    s = (f"{tag:58s} iters mean {it.mean():7.1f} p99 {np.percentile(it, 99):6.0f} max {it.max():6d} "
         f"opt {np.mean(r['status'] == 0):.3f} to1e-4 {tr[:, 1].mean():7.1f} to1e-5 {tr[:, 2].mean():7.1f} "
         f"wall {r['wall']:.1f}s")
    if base_obj is not None:
        s += f" maxrel {np.max(np.abs(r['obj'] - base_obj) / np.maximum(np.abs(base_obj), 1.0)):.1e}"
    print(s, flush=True)


def main():
    S = int(sys.argv[1])
    variants = [json.loads(v) for v in sys.argv[2:]] or [{}]
    mode = os.environ.get("LAB_MODE", "both")
    groups = scenarios.config4(range(S))
    wins = [[lp for lp in builder.group_window_lps(g)] for g in groups]  # [window id][scenario]
    P = scenarios.sweep_parameters(range(S))
    stride = int(os.environ.get("LAB_STRIDE", "32"))
    feats = scenarios.sweep_features(P)
    extra = os.environ.get("LAB_FEAT", "")
    cols = {"price": P["price_scale"], "demand": P["demand"], "rte": P["rte"], "load": np.log(P["load_scale"]),
            "E": np.log(P["E"])}
    for name in [e for e in extra.split(",") if e]:
        wgt = 1.0
        if ":" in name:
            name, wgt = name.split(":")[0], float(name.split(":")[1])
        col = cols[name]
        feats = np.concatenate([feats, (wgt * (col - col.mean()) / col.std())[:, None]], axis=1)
    seeds, rest, pick = seed_split(P["E"], stride, feats)
    warm_mode = os.environ.get("LAB_WARM", "nearest")
    if warm_mode.startswith("avg") or warm_mode.startswith("idw") or warm_mode.startswith("lin"):
        # the q nearest seeds in standardised features; lin<q>l<lam>: IDW weights moved toward the affine combination
        # that reproduces the window's own features (min |F'w - f|^2 + lam |w - w_idw|^2, sum w = 1)
        lam = float(warm_mode.split("l")[-1]) if warm_mode.startswith("lin") else 0.0
        q = int(warm_mode[3:].split("p")[0].split("l")[0])
        pw_ = float(warm_mode.split("p")[1]) if "p" in warm_mode[3:] else 1.0
        f = feats
        f = (f - f.mean(0)) / np.where(f.std(0) > 0, f.std(0), 1.0)
        d = ((f[rest][:, None, :] - f[seeds][None, :, :]) ** 2).sum(-1)
        pick2 = np.argsort(d, axis=1)[:, :q]
        dd = np.sqrt(np.take_along_axis(d, pick2, 1))
        wgt = np.full(dd.shape, 1.0 / q) if warm_mode.startswith("avg") else \
            (1.0 / np.maximum(dd, 1e-9) ** pw_) / (1.0 / np.maximum(dd, 1e-9) ** pw_).sum(1, keepdims=True)
        if warm_mode.startswith("lin"):
            one = np.ones(q)
            for i in range(len(rest)):
                F = f[seeds][pick2[i]]  # [q, d]
                A = F @ F.T + lam * np.eye(q)
                rhs = F @ f[rest[i]] + lam * wgt[i]
                ai, a1 = np.linalg.solve(A, rhs), np.linalg.solve(A, one)
                wgt[i] = ai - (one @ ai - 1.0) / (one @ a1) * a1
    lab = Lab()
    ref = None
    for v in variants:
        env = {k: v[k] for k in v if k.startswith("LAB_")}
        opts = {k: v[k] for k in v if not k.startswith("LAB_")}
        for k in list(os.environ):
            if k.startswith("LAB_") and k != "LAB_MODE":
                del os.environ[k]
        os.environ.update({k: str(x) for k, x in env.items()})
        tag = json.dumps(v)
        if mode in ("both", "cold"):
            lps = [lp for w in wins for lp in w]
            r = lab.solve(lps, check_every=opts.pop("cold_check", 32), kkt_every=1, **opts)
            if ref is None:
                ref = r["obj"]
            summary("cold " + tag, r, ref)
        if mode in ("both", "warm"):
            wo = dict(opts)
            seed_lps = [w[s] for w in wins for s in seeds]
            rs = lab.solve(seed_lps, check_every=32, kkt_every=1, **wo)
            ns = len(seeds)
            starts, lps = [], []
            for wi, w in enumerate(wins):
                for i, s in enumerate(rest):
                    k = wi * ns + pick[i]
                    lps.append(w[s])
                    if warm_mode != "nearest":
                        a = [transfer(w[s], seed_lps[wi * ns + p], rs["x"][wi * ns + p], rs["y"][wi * ns + p])
                             for p in pick2[i]]
                        starts.append((sum(wq * aa[0] for wq, aa in zip(wgt[i], a)),
                                       sum(wq * aa[1] for wq, aa in zip(wgt[i], a))))
                    else:
                        starts.append(transfer(w[s], seed_lps[k], rs["x"][k], rs["y"][k]))
            pw_in = None
            pwt = int(env.get("LAB_PWT", 0))
            if pwt and warm_mode != "nearest":  # the partners' final primal weights (mode 1) or final / data ratios (2)
                src = rs["pw"] if pwt == 1 else rs["pw"] / rs["pw0"]
                pw_in = []
                for wi in range(len(wins)):
                    for i in range(len(rest)):
                        pw_in.append(float(np.exp(sum(wq * np.log(src[wi * ns + p]) for wq, p in zip(wgt[i], pick2[i])))))
            r = lab.solve(lps, starts, pw_in=pw_in, check_every=64, kkt_every=1, warm_start=1, **wo)
            summary("warm " + tag, r)


if __name__ == "__main__":
    main()
