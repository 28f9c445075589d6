"""TEST INFRASTRUCTURE, never shipped: an independent pure-Python restatement
of docs/SEMANTICS.md, the second opinion on the C oracle (SURVEY.md §4 test
plan 3, §7 step 3, §8(c)).

It is written from the normative text alone, as straight-line scenario-at-a-
time code with Python integers and floats (binary64, the operation order the
text writes), sharing nothing with oracle/ccka_oracle.c or the HIP engine but
the input structures (ccka.world WorldSpec / ScenarioSet, ccka.abi structs).
tests/test_spec_model.py compares it with the C oracle on random small worlds
(hypothesis). Reference anchors are those of SEMANTICS.md: profile patches
demo_19_reset_policies.sh:68-75, demo_20_offpeak_configure.sh:59-81,
demo_21_peak_configure.sh:56-77; demand demo_30_burst_configure.sh:57-141;
PDB demo_10_setup_configure.sh:47-56; k8s 1.34 (.env:4), Karpenter 1.8.1
(05_karpenter.sh:20).

Scope: every section of SEMANTICS §3 for HPA, KEDA (one trigger) and static
deployments, including the HPA sync sub-steps, pool limits, drift (G0) and
replacement consolidation (G2); multi-node consolidation (G3) and extra KEDA
triggers are not restated here.
"""
from __future__ import annotations

import math

from ccka import abi

STEP = abi.STEP_SECONDS
SPOT, OD = abi.CAP_SPOT, abi.CAP_OD


def cap_bit(c):
    return SPOT if c == 0 else OD


def tdiv(a, b):
    """C truncating integer division."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def int32_ceil(x):
    return int(math.ceil(x))


class Node:
    __slots__ = ("used", "pool", "type", "zone", "cap", "ready_step", "last_event", "pods", "src")

    def __init__(self, D):
        self.used = False
        self.pool = self.type = self.zone = self.cap = 0
        self.ready_step = self.last_event = 0
        self.pods = [0] * D
        self.src = 0  # bit mask of the slots this node replaces (in-flight replacement)


class Scenario:
    """One scenario's rollout (SEMANTICS §2/§3)."""

    def __init__(self, spec, sc, s, load):
        self.spec = spec
        self.T = spec.n_steps
        self.D = len(spec.deploys)
        self.N = spec.max_nodes
        self.types = spec.catalog.itypes()
        self.K = spec.catalog.k
        self.Z = spec.n_zones
        self.price = spec.price
        self.ci_gpwh = spec.ci / 1000.0
        self.ci_gpwmin = spec.ci / 60000.0
        self.deps = list(spec.deploys)
        gid = sc.first_id + s
        self.col = gid % sc.n_traces if sc.n_traces > 0 else s
        self.load = load

        def ov(name, default):
            a = getattr(sc, name)
            return default if a is None else a[s].item()

        self.region = ov("region", 0)
        self.target = [ov("target_util_pct", d.target_util_pct) if d.scaler == abi.SCALER_HPA else d.target_util_pct
                       for d in self.deps]
        self.maxr = [ov("max_replicas", d.max_replicas) if d.scaler == abi.SCALER_HPA else d.max_replicas
                     for d in self.deps]
        self.down_w = [ov("down_stab_s", d.down.stab_window_s) if d.scaler == abi.SCALER_HPA else d.down.stab_window_s
                       for d in self.deps]
        self.cap_sel = [ov("cap_sel", d.cap_sel) for d in self.deps]
        self.reset_ca = ov("reset_ca_s", spec.reset_ca_s)
        self.switch = ov("peak_switch", spec.peak_switch)
        self.cw1000 = ov("carbon_weight", spec.carbon_weight) * 1000.0
        self.sync = spec.hpa_sync_s if spec.hpa_sync_s not in (0, STEP) else STEP
        self.S = STEP // self.sync
        # §1: pools start as base spec + RESET (its consolidateAfter is reset_ca_s)
        self.pools = []
        for p in spec.pools:
            st = {"policy": 0, "ca": 0, "zm": 0, "cm": 0}
            self.patch(st, p.base, None)
            self.patch(st, p.profile[abi.PROFILE_RESET], self.reset_ca)
            self.pools.append(st)
        self.profile = None
        self.nodes = [Node(self.D) for _ in range(self.N)]
        self.replicas = [d.replicas0 for d in self.deps]
        self.hist = [[] for _ in self.deps]  # per deployment: entries (rec, valid, delta), newest last
        self.last_active = [0] * self.D
        self.util = [None] * self.D
        self.kact = [False] * self.D
        self.cost = self.pend_min = self.energy_nw = self.e_hour = 0
        self.gco2 = 0.0
        self.slo = self.nmin_spot = self.nmin_od = self.launches = self.deletions = self.peak_nodes = 0
        self.last_choice = 0xFFFFFFFF
        self.hash = 2166136261
        self.prev_hour = None
        self.traj = []

    # ------------------------------------------------------------------ A
    @staticmethod
    def patch(st, x, ca_override):
        if x.policy:
            st["policy"] = x.policy
        if x.consolidate_after_s >= 0:
            st["ca"] = x.consolidate_after_s if ca_override is None else ca_override
        if x.zone_mask:
            st["zm"] = x.zone_mask
        if x.cap_mask:
            st["cm"] = x.cap_mask

    def in_window(self, minute):
        s, e = self.spec.peak_start, self.spec.peak_end
        return (s <= minute < e) if s <= e else (minute >= s or minute < e)

    # ------------------------------------------------------------------ helpers
    def ready(self, n, t):
        nd = self.nodes[n]
        return nd.used and nd.ready_step <= t

    def ready_pods(self, d, t):
        return sum(nd.pods[d] for n, nd in enumerate(self.nodes) if self.ready(n, t))

    def placed(self, d):
        return sum(nd.pods[d] for nd in self.nodes if nd.used)

    def usage(self, nd):
        c = m = p = 0
        for d, dep in enumerate(self.deps):
            c += nd.pods[d] * dep.req_cpu_m
            m += nd.pods[d] * dep.req_mem_mi
            p += nd.pods[d]
        return c, m, p

    def fit_type(self, ty, uc, um, up, d):
        """max additional pods of deployment d on type ty holding (uc, um, up); -1 if it cannot hold them"""
        if uc > ty.alloc_cpu_m or um > ty.alloc_mem_mi or up > ty.max_pods:
            return -1
        f = ty.max_pods - up
        dep = self.deps[d] if d is not None else None
        if dep is not None and dep.req_cpu_m > 0:
            f = min(f, (ty.alloc_cpu_m - uc) // dep.req_cpu_m)
        if dep is not None and dep.req_mem_mi > 0:
            f = min(f, (ty.alloc_mem_mi - um) // dep.req_mem_mi)
        return f

    def node_fit(self, nd, d):
        return max(self.fit_type(self.types[nd.type], *self.usage(nd), d), 0)

    def tainted(self, n):
        if self.nodes[n].src:
            return True
        return any(m.used and (m.src >> n & 1) for m in self.nodes)

    def node_price(self, nd, hr):
        return int(self.price[self.region, hr, nd.type, nd.zone, nd.cap])

    def pool_use(self, q):
        cpu = mem = 0
        for nd in self.nodes:
            if nd.used and nd.pool == q:
                cpu += self.types[nd.type].vcpu * 1000
                mem += self.types[nd.type].mem_mi
        return cpu, mem

    def limits_ok(self, q, use, ty):
        p = self.spec.pools[q]
        if p.limit_cpu_m >= 0 and use[0] + ty.vcpu * 1000 > p.limit_cpu_m:
            return False
        if p.limit_mem_mi >= 0 and use[1] + ty.mem_mi > p.limit_mem_mi:
            return False
        return True

    def offered(self, k, hr, zm, cm, c_only=None):
        for z in range(self.Z):
            if not (zm >> z & 1):
                continue
            for c in (0, 1):
                if c_only is not None and c != c_only:
                    continue
                if (cm & cap_bit(c)) and self.price[self.region, hr, k, z, c] > 0:
                    return True
        return False

    def free_slot(self):
        for n, nd in enumerate(self.nodes):
            if not nd.used:
                return n
        return -1

    def launch_choice(self, q, hr, zm, cm, sums, use):
        """SEMANTICS 3.F launch rule: (k, z, c, price) or None"""
        cands = [k for k in range(self.K)
                 if self.fit_type(self.types[k], *sums, None) >= 0 and self.limits_ok(q, use, self.types[k])]
        spot_only = bool(cm & SPOT) and any(self.offered(k, hr, zm, SPOT, 0) for k in cands)
        best = None
        for k in cands:
            for z in range(self.Z):
                if not (zm >> z & 1):
                    continue
                for c in (0, 1):
                    if not (cm & cap_bit(c)) or (spot_only and c != 0):
                        continue
                    pr = int(self.price[self.region, hr, k, z, c])
                    if pr <= 0:
                        continue
                    score = float(pr) + self.cw1000 * (self.types[k].p_ref_w * self.ci_gpwh[self.region, hr])
                    key = (score, k, z, c)
                    if best is None or key < best[0]:
                        best = (key, pr)
        if best is None:
            return None
        (_, k, z, c), pr = best
        return k, z, c, pr

    def offer(self, q, hr, zm, cm, sums, use):
        """SEMANTICS 3.G2 offer rule: the lexicographic minimum of (price, k, z, c)"""
        best = None
        for k in range(self.K):
            ty = self.types[k]
            if self.fit_type(ty, *sums, None) < 0 or not self.limits_ok(q, use, ty):
                continue
            for z in range(self.Z):
                if not (zm >> z & 1):
                    continue
                for c in (0, 1):
                    if not (cm & cap_bit(c)):
                        continue
                    pr = int(self.price[self.region, hr, k, z, c])
                    if pr > 0 and (best is None or (pr, k, z, c) < best):
                        best = (pr, k, z, c)
        if best is None:
            return None
        pr, k, z, c = best
        return k, z, c, pr

    def launch(self, slot, q, k, z, c, t, pods, src=0):
        nd = self.nodes[slot]
        nd.used = True
        nd.pool, nd.type, nd.zone, nd.cap = q, k, z, c
        nd.ready_step = t + self.spec.provision_delay_steps
        nd.last_event = t
        nd.pods = list(pods)
        nd.src = src
        self.launches += 1
        self.last_choice = k | z << 12 | c << 14 | q << 16
        self.hash = ((self.hash ^ self.last_choice) * 16777619) & 0xFFFFFFFF
        self.step_last_type = k

    def free(self, n):
        self.nodes[n] = Node(self.D)
        for m in self.nodes:
            m.src &= ~(1 << n)

    # ------------------------------------------------------------------ C
    def window(self, d, W):
        """entries inside a window / period of W seconds, newest first"""
        h = self.hist[d]
        out = []
        for k in range(len(h)):
            if (k + 1) * self.sync < W:
                out.append(h[len(h) - 1 - k])
        return out

    def behavior(self, d, proposal, cur, lo, hi):
        dep = self.deps[d]
        up_recs = [e[0] for e in self.window(d, dep.up.stab_window_s) if e[1]]
        dn_recs = [e[0] for e in self.window(d, self.down_w[d]) if e[1]]
        up = min([proposal] + up_recs)
        down = max([proposal] + dn_recs)
        rec = max(cur, up)
        rec = min(rec, down)

        def limit(rules, is_up):
            if rules.select == abi.SELECT_DISABLED or rules.n_policies == 0:
                return cur
            vals = []
            for q in range(rules.n_policies):
                pol = rules.policies[q]
                ent = self.window(d, pol.period_s)
                added = sum(max(e[2], 0) for e in ent)
                removed = sum(max(-e[2], 0) for e in ent)
                ps = cur - added + removed
                if pol.type == abi.HPA_PODS:
                    vals.append(ps + pol.value if is_up else ps - pol.value)
                elif is_up:
                    vals.append(int32_ceil(float(ps) * (1.0 + float(pol.value) / 100.0)))
                else:
                    vals.append(int(float(ps) * (1.0 - float(pol.value) / 100.0)))
            if is_up:
                return max(vals) if rules.select == abi.SELECT_MAX else min(vals)
            return min(vals) if rules.select == abi.SELECT_MAX else max(vals)

        if rec > cur:
            hi = min(hi, max(limit(dep.up, True), cur))
        elif rec < cur:
            lo = max(lo, min(limit(dep.down, False), cur))
        return lo if rec < lo else (hi if rec > hi else rec)

    def within(self, d, x):
        tol = self.deps[d].tolerance
        return 1.0 - tol <= x <= 1.0 + tol

    def hpa_decide(self, d, t, L, ready):
        dep = self.deps[d]
        cur = self.replicas[d]
        minr, maxr = dep.min_replicas, self.maxr[d]
        self.util[d] = None  # the SLO reads the step's last decision's utilisation
        if cur == 0 and minr != 0:
            self.hist[d].append((0, False, 0))
            return
        if cur > maxr or cur < minr or ready == 0:
            desired = maxr if cur > maxr else (minr if cur < minr else cur)
            self.hist[d].append((0, False, desired - cur))
            self.replicas[d] = desired
            return
        usage = L if dep.limit_cpu_m <= 0 else min(L, ready * dep.limit_cpu_m)
        util = tdiv(usage * 100, ready * dep.req_cpu_m)
        self.util[d] = util
        target = self.target[d]
        ratio = float(util) / float(target)
        if cur - ready > 0 and ratio > 1.0:
            nutil = tdiv(usage * 100, cur * dep.req_cpu_m)
            nr = float(nutil) / float(target)
            if self.within(d, nr) or nr < 1.0:
                proposal = cur
            else:
                proposal = max(int32_ceil(nr * float(cur)), cur)
        else:
            proposal = cur if self.within(d, ratio) else int32_ceil(ratio * float(ready))
        desired = self.behavior(d, proposal, cur, minr, maxr)
        self.hist[d].append((proposal, True, desired - cur))
        self.replicas[d] = desired

    def keda_decide(self, d, t, L):
        dep = self.deps[d]
        cur = self.replicas[d]
        active = L > dep.keda_activation
        self.kact[d] = active
        if active:
            self.last_active[d] = t
        if cur == 0:
            self.hist[d].append((0, False, 0))
            self.replicas[d] = 1 if active else 0
            return
        if not active and dep.keda_min == 0 and STEP * (t - self.last_active[d]) >= dep.keda_cooldown_s:
            self.hist[d].append((0, False, 0))
            self.replicas[d] = 0
            return
        minr, maxr = max(dep.keda_min, 1), dep.keda_max
        if cur > maxr or cur < minr:
            desired = maxr if cur > maxr else minr
            self.hist[d].append((0, False, desired - cur))
            self.replicas[d] = desired
            return
        thr = dep.keda_threshold
        r = float(L) / (float(thr) * float(cur))
        proposal = cur if self.within(d, r) else int32_ceil(float(L) / float(thr))
        desired = self.behavior(d, proposal, cur, minr, maxr)
        self.hist[d].append((proposal, True, desired - cur))
        self.replicas[d] = desired

    # ------------------------------------------------------------------ step
    def first_fit(self, d, count, slots, t, apply=True):
        """place `count` pods of d first-fit over `slots` (slot order); returns the rest"""
        for n in slots:
            if count <= 0:
                break
            nd = self.nodes[n]
            if not (cap_bit(nd.cap) & self.cap_sel[d]):
                continue
            k = min(count, self.node_fit(nd, d))
            if k > 0:
                if apply:
                    nd.pods[d] += k
                    nd.last_event = t
                count -= k
        return count

    def step(self, t):
        minute = (self.spec.start_minute + t) % 1440
        hr = minute // 60
        flags = 0
        self.step_last_type = 0xFFFF
        if self.prev_hour is not None and hr != self.prev_hour:  # H: the carbon of the hour that ended
            self.gco2 += float(self.e_hour) * (self.ci_gpwmin[self.region, self.prev_hour] * 1e-9)
            self.e_hour = 0
        self.prev_hour = hr
        # A. profile
        peak = bool(self.switch) and self.in_window(minute)
        prof = abi.PROFILE_PEAK if peak else abi.PROFILE_OFFPEAK
        if peak:
            flags |= 1
        if prof != self.profile:
            self.profile = prof
            for q, p in enumerate(self.spec.pools):
                self.patch(self.pools[q], p.profile[prof], None)
        # C. scalers
        for d, dep in enumerate(self.deps):
            if dep.scaler not in (abi.SCALER_HPA, abi.SCALER_KEDA):
                continue
            L = int(self.load[t, d, self.col])
            ready = self.ready_pods(d, t)
            self.util[d] = None
            for _ in range(self.S):
                if dep.scaler == abi.SCALER_HPA:
                    self.hpa_decide(d, t, L, ready)
                else:
                    self.keda_decide(d, t, L)
        # D. ReplicaSet reconcile: nominated first, then running, high slot first
        for d in range(self.D):
            excess = self.placed(d) - self.replicas[d]
            for want_ready in (False, True):
                for n in range(self.N - 1, -1, -1):
                    nd = self.nodes[n]
                    if excess <= 0 or not nd.used or self.ready(n, t) != want_ready:
                        continue
                    k = min(nd.pods[d], excess)
                    if k > 0:
                        nd.pods[d] -= k
                        nd.last_event = t
                        excess -= k
        # E. kube-scheduler (ready slots), F1. nomination (in-flight slots)
        for want_ready in (True, False):
            for d in range(self.D):
                p = self.replicas[d] - self.placed(d)
                if p > 0:
                    slots = [n for n in range(self.N)
                             if self.nodes[n].used and self.ready(n, t) == want_ready and not self.tainted(n)]
                    self.first_fit(d, p, slots, t)
        # F2. Karpenter NodeClaims
        self.provision(t, hr)
        flags |= 2 if self.step_last_type != 0xFFFF else 0
        # G. disruption
        flags |= self.disrupt(t, hr)
        # H. accounting
        flags |= self.account(t, hr)
        used = [nd for nd in self.nodes if nd.used]
        nsp = sum(1 for nd in used if nd.cap == 0)
        nod = len(used) - nsp
        pending = sum(self.replicas[d] - self.ready_pods(d, t) for d in range(self.D))
        self.traj.append((sum(self.replicas), pending, nsp, nod, self.step_last_type, flags))

    def claim_j(self, q, hr, zm, cm, sums, d, use):
        best = 0
        for k in range(self.K):
            ty = self.types[k]
            if not self.limits_ok(q, use, ty) or not self.offered(k, hr, zm, cm):
                continue
            f = self.fit_type(ty, *sums, d)
            if f > best:
                best = f
        return best

    def provision(self, t, hr):
        order = sorted(range(self.D), key=lambda d: (-self.deps[d].req_cpu_m, -self.deps[d].req_mem_mi, d))
        start_use = [self.pool_use(q) for q in range(len(self.pools))]
        claims = []
        reserved = set()
        for d in order:
            dep = self.deps[d]
            pending = self.replicas[d] - self.placed(d) - sum(cl["pods"][d] for cl in claims)
            if pending <= 0:
                continue
            for cl in claims:
                if pending <= 0:
                    break
                cm = cl["cm"] & self.cap_sel[d]
                if not cm:
                    continue
                j = self.claim_j(cl["q"], hr, cl["zm"], cm, cl["sums"], d, start_use[cl["q"]])
                if j <= 0:
                    continue
                k = min(pending, j)
                cl["cm"] = cm
                c0, m0, p0 = cl["sums"]
                cl["sums"] = (c0 + k * dep.req_cpu_m, m0 + k * dep.req_mem_mi, p0 + k)
                cl["pods"][d] += k
                pending -= k
            # new claims in the first pool (Karpenter order) that admits the
            # deployment's capacity types and can hold a pod of it (j > 0: an
            # offered type within the pool's limits at step start)
            q, j = None, 0
            for qq in range(len(self.pools)):
                cm = self.pools[qq]["cm"] & self.cap_sel[d]
                if cm:
                    j = self.claim_j(qq, hr, self.pools[qq]["zm"], cm, (0, 0, 0), d, start_use[qq])
                    if j > 0:
                        q = qq
                        break
            if q is None:
                continue
            while pending > 0:
                slot = next((n for n in range(self.N) if not self.nodes[n].used and n not in reserved), None)
                if slot is None:
                    break
                zm, cm = self.pools[q]["zm"], self.pools[q]["cm"] & self.cap_sel[d]
                k = min(pending, j)
                pods = [0] * self.D
                pods[d] = k
                claims.append({"q": q, "zm": zm, "cm": cm, "slot": slot, "pods": pods,
                               "sums": (k * dep.req_cpu_m, k * dep.req_mem_mi, k)})
                reserved.add(slot)
                pending -= k
        for cl in claims:
            q = cl["q"]
            ch = self.launch_choice(q, hr, cl["zm"], cl["cm"], cl["sums"], self.pool_use(q))
            if ch is None:
                continue  # dropped: the slot stays free, the pods pending
            k, z, c, _ = ch
            self.launch(cl["slot"], q, k, z, c, t, cl["pods"])

    def pdb_allowed(self, t):
        pct = self.spec.pdb_pct
        if pct < 0:
            return None
        rdy = sum(self.ready_pods(d, t) for d in range(self.D) if self.deps[d].pdb_member)
        reps = sum(self.replicas[d] for d in range(self.D) if self.deps[d].pdb_member)
        return max(0, rdy - (pct * reps + 99) // 100)

    def pdb_pods(self, nd):
        return sum(nd.pods[d] for d in range(self.D) if self.deps[d].pdb_member)

    def drifted(self, nd):
        st = self.pools[nd.pool]
        return not (st["zm"] >> nd.zone & 1) or not (st["cm"] & cap_bit(nd.cap))

    def disrupt(self, t, hr):
        flags = 0
        drift_on = self.spec.drift
        # G1/G2 takeover: ready replacements take their sources' pods (sources in slot order)
        for m in range(self.N):
            nm = self.nodes[m]
            if not (nm.used and nm.src and self.ready(m, t)):
                continue
            srcs = [n for n in range(self.N) if nm.src >> n & 1]
            for n in srcs:
                ns = self.nodes[n]
                for d in range(self.D):
                    k = min(ns.pods[d], self.node_fit(nm, d)) if (cap_bit(nm.cap) & self.cap_sel[d]) else 0
                    nm.pods[d] += k
                nm.last_event = t
                nm.src &= ~(1 << n)
                self.free(n)
                self.deletions += 1
                flags |= 4
            nm.last_event = t
        allowed = self.pdb_allowed(t)
        for q, pool in enumerate(self.spec.pools):
            st = self.pools[q]
            npool = sum(1 for nd in self.nodes if nd.used and nd.pool == q)
            if npool == 0:
                continue
            budget = (pool.budget_pct * npool + 99) // 100
            deleted = 0
            # G0 drift
            if drift_on:
                for n in range(self.N):
                    if deleted >= budget:
                        break
                    nd = self.nodes[n]
                    if not (nd.used and nd.pool == q and self.ready(n, t) and self.drifted(nd)):
                        continue
                    if any(m.used and (m.src >> n & 1) for m in self.nodes):
                        continue  # already waiting for its replacement
                    pp = self.pdb_pods(nd)
                    if allowed is not None and pp > allowed:
                        continue
                    recv = [m for m in range(self.N) if m != n and self.nodes[m].used and self.ready(m, t)
                            and not self.drifted(self.nodes[m]) and not self.tainted(m)]
                    left = [0] * self.D
                    for d in range(self.D):
                        left[d] = self.first_fit(d, nd.pods[d], recv, t)
                    nd.pods = left
                    slot = self.free_slot()
                    ch = None
                    if sum(left) > 0 and slot >= 0:
                        cm = st["cm"]
                        for d in range(self.D):
                            if left[d] > 0:
                                cm &= self.cap_sel[d]
                        sums = (sum(left[d] * self.deps[d].req_cpu_m for d in range(self.D)),
                                sum(left[d] * self.deps[d].req_mem_mi for d in range(self.D)), sum(left))
                        if cm:
                            ch = self.launch_choice(q, hr, st["zm"], cm, sums, self.pool_use(q))
                    if sum(left) > 0 and ch is not None:
                        k, z, c, _ = ch
                        self.launch(slot, q, k, z, c, t, [0] * self.D, src=1 << n)
                        flags |= 2 | 16 | 32
                    else:
                        self.free(n)
                        self.deletions += 1
                        flags |= 4 | 16
                    if allowed is not None:
                        allowed -= pp
                    deleted += 1
            # consolidation
            while deleted < budget:
                cands = []
                for n in range(self.N):
                    nd = self.nodes[n]
                    if not (nd.used and nd.pool == q and self.ready(n, t)) or self.tainted(n):
                        continue
                    if STEP * (t - nd.last_event) < st["ca"]:
                        continue
                    cands.append((sum(nd.pods), -self.node_price(nd, hr), n))
                cands.sort()
                chosen = None
                for pods, _, n in cands:
                    nd = self.nodes[n]
                    if pods == 0:
                        chosen = n
                        break
                    if st["policy"] != abi.WHEN_EMPTY_OR_UNDERUTILIZED:
                        continue
                    if allowed is not None and self.pdb_pods(nd) > allowed:
                        continue
                    recv = [m for m in range(self.N) if m != n and self.nodes[m].used and self.ready(m, t)
                            and not self.tainted(m)]
                    # trial first-fit on copies
                    saved = [(list(self.nodes[m].pods), self.nodes[m].last_event) for m in range(self.N)]
                    ok = all(self.first_fit(d, nd.pods[d], recv, t, apply=True) == 0 for d in range(self.D))
                    for m in range(self.N):
                        self.nodes[m].pods, self.nodes[m].last_event = saved[m]
                    if ok:
                        chosen = n
                        break
                if chosen is None:
                    break
                nd = self.nodes[chosen]
                recv = [m for m in range(self.N) if m != chosen and self.nodes[m].used and self.ready(m, t)
                        and not self.tainted(m)]
                if allowed is not None:
                    allowed -= self.pdb_pods(nd)
                for d in range(self.D):
                    self.first_fit(d, nd.pods[d], recv, t)
                self.free(chosen)
                self.deletions += 1
                deleted += 1
                flags |= 4
            # G2 replacement offer
            if self.spec.replace and st["policy"] == abi.WHEN_EMPTY_OR_UNDERUTILIZED and deleted < budget:
                cands = []
                for n in range(self.N):
                    nd = self.nodes[n]
                    if not (nd.used and nd.pool == q and self.ready(n, t) and nd.cap == 1 and sum(nd.pods) > 0):
                        continue
                    if STEP * (t - nd.last_event) < st["ca"]:
                        continue
                    if any(m.used and (m.src >> n & 1) for m in self.nodes) or nd.src:
                        continue
                    cands.append((sum(nd.pods), -self.node_price(nd, hr), n))
                cands.sort()
                for pods, negp, n in cands:
                    nd = self.nodes[n]
                    slot = self.free_slot()
                    if slot < 0:
                        break
                    if allowed is not None and self.pdb_pods(nd) > allowed:
                        continue
                    cm = st["cm"]
                    for d in range(self.D):
                        if nd.pods[d] > 0:
                            cm &= self.cap_sel[d]
                    if not cm:
                        continue
                    ch = self.offer(q, hr, st["zm"], cm, self.usage(nd), self.pool_use(q))
                    if ch is None or ch[3] >= -negp:
                        continue
                    k, z, c, _ = ch
                    self.launch(slot, q, k, z, c, t, [0] * self.D, src=1 << n)
                    flags |= 2 | 32
                    deleted += 1
                    break
        return flags

    def account(self, t, hr):
        flags = 0
        r = self.region
        bt = self.types[self.spec.catalog.index(self.spec.base_type)]
        cost = self.spec.base_nodes * int(self.price[r, hr, self.spec.catalog.index(self.spec.base_type), 0, 1])
        base_nw = self.spec.base_nodes * (bt.idle_nw + bt.dyn_nw_per_m * int(self.spec.base_util * float(bt.alloc_cpu_m)))
        upp = []
        for d, dep in enumerate(self.deps):
            rd = self.ready_pods(d, t)
            L = int(self.load[t, d, self.col])
            if rd > 0:
                u = max(0, L if dep.limit_cpu_m <= 0 else min(L, rd * dep.limit_cpu_m))
                upp.append(tdiv(u, rd))
            else:
                upp.append(0)
        e = base_nw
        for n, nd in enumerate(self.nodes):
            if not nd.used:
                continue
            ty = self.types[nd.type]
            cost += self.node_price(nd, hr)
            use = min(sum(nd.pods[d] * upp[d] for d in range(self.D)), ty.alloc_cpu_m) if self.ready(n, t) else 0
            e += ty.idle_nw + ty.dyn_nw_per_m * use
        self.cost += cost
        self.energy_nw += e
        self.e_hour += e
        pending = sum(self.replicas[d] - self.ready_pods(d, t) for d in range(self.D))
        slo = pending > 0
        for d, dep in enumerate(self.deps):
            if dep.scaler == abi.SCALER_HPA and self.util[d] is not None and self.util[d] > self.spec.slo_util_pct:
                slo = True
            if dep.scaler == abi.SCALER_KEDA and self.kact[d] and self.replicas[d] == 0:
                slo = True
        if slo:
            self.slo += 1
            flags |= 8
        self.pend_min += pending
        used = [nd for nd in self.nodes if nd.used]
        self.nmin_spot += sum(1 for nd in used if nd.cap == 0)
        self.nmin_od += sum(1 for nd in used if nd.cap == 1)
        self.peak_nodes = max(self.peak_nodes, len(used))
        return flags

    def run(self):
        for t in range(self.T):
            self.step(t)
        if self.prev_hour is not None:
            self.gco2 += float(self.e_hour) * (self.ci_gpwmin[self.region, self.prev_hour] * 1e-9)
        return {
            "cost_uphmin": self.cost, "energy_wmin": float(self.energy_nw) * 1e-9, "gco2": self.gco2,
            "slo_minutes": self.slo, "pending_pod_minutes": self.pend_min, "node_min_spot": self.nmin_spot,
            "node_min_od": self.nmin_od, "launches": self.launches, "deletions": self.deletions,
            "peak_nodes": self.peak_nodes, "final_replicas": sum(self.replicas),
            "final_nodes": sum(1 for nd in self.nodes if nd.used), "last_choice": self.last_choice,
            "choice_hash": self.hash,
        }, self.traj


def rollout(spec, sc, load):
    """Every scenario of `sc` (load [T][D][columns]); returns (results dict of
    lists, trajectories [scenario][step] of record tuples)."""
    res, trajs = {}, []
    for s in range(sc.n):
        r, tr = Scenario(spec, sc, s, load).run()
        for k, v in r.items():
            res.setdefault(k, []).append(v)
        trajs.append(tr)
    return res, trajs
