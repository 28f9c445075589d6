"""Schedule model of rollout_d1_kernel's lane-skewed waves (analysis aid, not a
test): the oracle's config-2 trajectories give each scenario's event steps
(replica changes, launches/deletions, readiness, clock hours); the model
replays them through the wave schedule (event runs every K iterations for the
stalled lanes, S quiet steps per iteration, lanes at most `slack` steps ahead
of the slowest one) and reports iterations and event runs per wave.
usage: python tests/sched_model.py [scenarios]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import pyoracle as po  # noqa: E402
from ccka import configs  # noqa: E402
from parity import oracle  # noqa: E402

T = 1440


def event_steps(tc, delay, hours=True):
    rep = tc["replicas"].astype(np.int64)
    ev = np.zeros(rep.shape, bool)
    ev[0] = True
    ev[1:] |= rep[1:] != rep[:-1]
    ev |= (tc["flags"] & (2 | 4)) != 0
    if hours:
        ev[::60] = True
    t, n = np.where((tc["flags"] & 2) != 0)
    ev[np.minimum(t + delay, T - 1), n] = True
    return ev


def simulate(ev, slack=48, S=4, K=2, lpw=49):
    its, runs = [], []
    for w in range(ev.shape[1] // lpw):
        E = ev[:, w * lpw:(w + 1) * lpw]
        t = np.zeros(lpw, np.int64)
        stall = np.zeros(lpw, bool)
        it = r = 0
        while (t < T).any():
            if stall.any() and it % K == K - 1:
                r += 1
                t[stall] += 1
                stall[:] = False
            if not (t < T).any():
                it += 1
                break
            lim = t[t < T].min() + slack
            for _ in range(S):
                act = (t < T) & ~stall & (t < lim)
                hit = np.zeros(lpw, bool)
                hit[act] = E[np.minimum(t[act], T - 1), np.where(act)[0]]
                stall |= hit
                t[act & ~hit] += 1
            it += 1
        its.append(it)
        runs.append(r)
    return float(np.mean(its)), int(np.max(its)), float(np.mean(runs))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 49 * 30
    spec = configs.config2_world()
    sc = configs.hpa_scenarios(n)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, n)
    _, tc = oracle(spec, sc, load, traj=True, threads=8)
    e1 = event_steps(tc, spec.provision_delay_steps)
    e0 = event_steps(tc, spec.provision_delay_steps, hours=False)
    print(f"event lane-steps {e1.mean():.4f}; clock hours {1 - e0.sum() / e1.sum():.1%} of events")
    for name, kw, ev in [("base (S=4, K=2, slack 48)", {}, e1), ("slack 112", {"slack": 112}, e1),
                         ("no clock-hour events", {}, e0), ("K=1", {"K": 1}, e1), ("S=6", {"S": 6}, e1)]:
        m, mx, r = simulate(ev, **kw)
        print(f"{name:28s} iterations/wave mean {m:.1f} max {mx}  event runs/wave {r:.1f}")


if __name__ == "__main__":
    main()
