"""Cost model of pooling rollout_d1_kernel's event runs across the waves of a
block (analysis aid, not a test; VERDICT r3 "model it first").

The oracle's config-2 trajectories give every scenario's event steps
(tests/sched_model.py); they are replayed through two schedules:

* per-wave (the round-3 kernel): 49 lanes per wave, S quiet steps per
  iteration, an event run for the wave's stalled lanes every K iterations;
  a SIMD runs two waves, so its time is the sum of both waves' issue cycles.
* pooled: the block's 8 waves (two per SIMD, 392 scenarios) run in lockstep;
  every K iterations the block's stalled lanes are gathered into
  ceil(stalled / 64) event runs on distinct SIMDs (state moves through LDS);
  each cadence costs the busiest SIMD's load.

Issue costs (cycles of one SIMD, calibrated on profiles/round3/config2_stamps.txt):
Q per wave-iteration (quiet steps + loop + top), E(n) per event run of n lanes,
X per wave and cadence for the state exchange.
usage: python tools/pool_model.py [blocks] [Q] [E16] [E64] [X]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import sched_model as sm  # noqa: E402

T = 1440


def e_run(n, e16, e64):
    return e16 + (e64 - e16) * (min(n, 64) - 16) / 48.0


def per_wave(E, S=8, K=2, slack=48):
    """iterations, event runs and run sizes of one wave (sched_model's rule)"""
    lpw = E.shape[1]
    t = np.zeros(lpw, np.int64)
    stall = np.zeros(lpw, bool)
    it = 0
    runs = []
    while (t < T).any():
        if stall.any() and it % K == K - 1:
            runs.append(int(stall.sum()))
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
    return it, runs


def pooled(E, waves=8, S=8, K=2, slack=48, q=2650, e16=6000, e64=7200, x=1500, simds=4):
    """lockstep block: cycles of the busiest SIMD summed over cadences"""
    n = E.shape[1]
    lpw = n // waves
    t = np.zeros(n, np.int64)
    stall = np.zeros(n, bool)
    it = 0
    cyc = 0.0
    rot = 0
    sizes = []
    load = np.zeros(simds)
    while (t < T).any():
        live = (t < T)
        # quiet cost: every wave holding a live scenario (floating: all waves while any is live)
        nw = min(waves, int(np.ceil(live.sum() / 64.0)) if live.any() else 0)
        nw = waves if live.sum() > 0 else 0
        load += q * nw / simds
        if it % K == K - 1 and stall.any():
            s = int(stall.sum())
            r = int(np.ceil(s / 64.0))
            per = s / r
            for j in range(r):
                load[(rot + j) % simds] += e_run(per, e16, e64)
                sizes.append(per)
            rot = (rot + r) % simds
            load += x * waves / simds
            cyc += load.max()
            load[:] = 0
            t[stall] += 1
            stall[:] = False
        if not (t < T).any():
            it += 1
            break
        # ring slack per origin group of lpw scenarios
        for _ in range(S):
            act = (t < T) & ~stall
            tl = t.copy()
            for g in range(waves):
                sl = slice(g * lpw, (g + 1) * lpw)
                lv = t[sl][t[sl] < T]
                if lv.size:
                    act[sl] &= t[sl] < lv.min() + slack
            hit = np.zeros(n, bool)
            hit[act] = E[np.minimum(tl[act], T - 1), np.where(act)[0]]
            stall |= hit
            t[act & ~hit] += 1
        it += 1
    cyc += load.max()
    return it, cyc, sizes


def main():
    blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    q = float(sys.argv[2]) if len(sys.argv) > 2 else 2650
    e16 = float(sys.argv[3]) if len(sys.argv) > 3 else 6000
    e64 = float(sys.argv[4]) if len(sys.argv) > 4 else 7200
    x = float(sys.argv[5]) if len(sys.argv) > 5 else 1500
    lpw, waves = 49, 8
    n = blocks * waves * lpw
    import pyoracle as po
    from ccka import configs
    from parity import oracle
    spec = configs.config2_world()
    sc = configs.hpa_scenarios(n)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, n)
    _, tc = oracle(spec, sc, load, traj=True, threads=8)
    ev = sm.event_steps(tc, spec.provision_delay_steps)
    print(f"{n} scenarios, event lane-steps {ev.mean():.4f}; Q {q} E16 {e16} E64 {e64} X {x}")
    # per-wave: SIMD s runs waves w (block b) and w (block b+1): pair consecutive blocks' waves
    simd_cyc = []
    its = []
    rs = []
    for b in range(0, blocks):
        for w in range(waves):
            E = ev[:, (b * waves + w) * lpw:(b * waves + w + 1) * lpw]
            it, runs = per_wave(E)
            its.append(it)
            rs += runs
            simd_cyc.append(it * q + sum(e_run(r, e16, e64) for r in runs))
    simd_cyc = np.array(simd_cyc).reshape(-1, 2).sum(1)  # two waves per SIMD
    print(f"per-wave  K=2: iterations mean {np.mean(its):.1f} max {max(its)}; runs/wave {len(rs) / len(its):.1f} "
          f"lanes/run {np.mean(rs):.1f}; SIMD cycles mean {simd_cyc.mean():.0f} max {simd_cyc.max():.0f}")
    base = simd_cyc.max()
    for K in [int(k) for k in os.environ.get("KS", "2,3,4").split(",")]:
        cs, itp, sz = [], [], []
        for b in range(blocks):
            E = ev[:, b * waves * lpw:(b + 1) * waves * lpw]
            it, cyc, sizes = pooled(E, waves=waves, K=K, q=q, e16=e16, e64=e64, x=x)
            cs.append(cyc)
            itp.append(it)
            sz += sizes
        print(f"pooled    K={K}: iterations mean {np.mean(itp):.1f}; lanes/run {np.mean(sz):.1f}; "
              f"busiest-SIMD cycles mean {np.mean(cs):.0f} max {max(cs):.0f} -> {base / max(cs):.2f}x")


if __name__ == "__main__":
    main()
