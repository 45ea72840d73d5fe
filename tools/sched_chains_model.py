"""Symbolic model of p2p_sched_chains_kernel's time-aligned schedule (design check, CPU only).

Takes per-call decisions (current frame, rollback depth, advance, delivered frame) of one session
from the oracle (oracle_p2p_sched_run's per-call rb_frame / advanced under an arrival schedule),
then
  * replays them sequentially (the reference's order: load, replay with saves, own save + advance),
  * and through the kernel's tables (lineage slot 0, chains on slots 1..15, last-writer masks,
    'holds the state before the exchange', hand-offs, ring sources) one time step per frame,
with states as hashes of (previous state, input), and checks that the final state and every ring
cell agree.  Usage: python tools/sched_chains_model.py [sessions] [calls] [max_prediction]
"""
import sys

import numpy as np

from oracle import oracle as o
from ggrs_amd import synth


def advance(st, h, inp):
    return hash((st, h, inp)) & 0xFFFFFFFFFFFF


def inputs_of(rows, h, dlv):
    """remote input of frame h as a call with delivered frame dlv sees it (repeat-last)."""
    if dlv < 0:
        return 0
    return int(rows[min(h, dlv)])


def sequential(calls, rows, R, launch):
    """calls: list of (cur, d, adv, dlv).  Returns the cell contents / frames and the cur state
    after each launch boundary (launch = list of call counts)."""
    ring = {}          # slot -> (frame, state)
    st = 0             # state at frame 0
    cells = {}
    for k, (cur, d, adv, dlv) in enumerate(calls):
        if cur == 0 and k == 0:
            ring[0] = (0, st)
        if d:
            m = cur - d
            fr, s = ring[m % R]
            assert fr == m, (k, m, fr)
            for h in range(m, cur):
                ring[h % R] = (h, s)
                s = advance(s, h, inputs_of(rows, h, dlv))
            st = s
        ring[cur % R] = (cur, st)
        if adv:
            st = advance(st, cur, inputs_of(rows, cur, dlv))
    return st, ring


def time_aligned(calls, rows, R, maxp, stages, st0=0, ring0=None, cur0=0):
    """The kernel's tables and step loop over one launch of calls (stage boundaries `stages`)."""
    NS = 16
    ring = dict(ring0 or {})
    tab = {}            # frame -> dict
    until = [-10 ** 9] * NS
    rrp = 0
    own_hi = cur0 - 1
    minpre = 10 ** 9
    for f in range(max(0, cur0 - maxp), cur0):
        tab[f] = dict(valid=0, adv=0, dlv=-1, lw=31, hold=16, hand=0, ch=[])
    ranges = []
    started, tn = False, 0
    ci = 0
    for si, K in enumerate(stages):
        last = si == len(stages) - 1
        for c in range(ci, ci + K):
            cur, d, adv, dlv = calls[c]
            if cur > own_hi:
                tab[cur] = dict(valid=1, adv=0, dlv=-1, lw=0, hold=0, hand=0, ch=[])
                own_hi = cur
            e = tab[cur]
            e["dlv"], e["adv"] = dlv, adv
            if d:
                m = cur - d
                slot = 0
                for k in range(1, NS):
                    j = 1 + (rrp + k - 1) % (NS - 1)
                    if until[j] <= m:
                        slot = j
                        break
                assert slot, "out of slots"
                rrp = slot
                until[slot] = cur
                assert len(tab[m]["ch"]) < 2
                tab[m]["ch"].append(dict(slot=slot, src=tab[m]["hold"], dlv=dlv, d=d))
                for h in range(m, cur + 1):
                    if h < cur:
                        tab[h]["lw"] = slot
                    if h > m:
                        tab[h]["hold"] = slot
                    if h == cur:
                        tab[h]["hand"] = slot
                if m < cur0:
                    minpre = min(minpre, m)
        ci += K
        cur_after = calls[ci][0] if ci < len(calls) else None
        T = own_hi + 1 if last else cur_after - maxp
        if not started and (last or T >= cur0):
            started, tn = True, min(cur0, minpre)
        rg = (tn, max(tn, T)) if started else (0, 0)
        if started:
            tn = rg[1]
        ranges.append(rg)
    # steps
    lanes = [None] * NS
    lanes[0] = st0
    act = [False] * NS
    cend = [0] * NS
    cdlv = [0] * NS
    for (tb, te) in ranges:
        for tau in range(tb, te):
            e = tab[tau]
            src = list(range(NS))
            ring_ld = [False] * NS
            for ch in e["ch"]:
                j = ch["slot"]
                act[j] = True
                cend[j] = tau + ch["d"]
                cdlv[j] = ch["dlv"]
                if ch["src"] == 16:
                    ring_ld[j] = True
                else:
                    src[j] = ch["src"]
            if e["valid"] and e["hand"]:
                src[0] = e["hand"]
            lanes = [lanes[src[j]] for j in range(NS)]
            for j in range(NS):
                if ring_ld[j]:
                    fr, s = ring[tau % R]
                    assert fr == tau, (tau, fr)
                    lanes[j] = s
            for j in range(NS):
                own = j == 0 and e["valid"]
                rep = j != 0 and act[j] and tau < cend[j]
                if (own or rep) and e["lw"] == j:
                    ring[tau % R] = (tau, lanes[j])
                if rep or (own and e["adv"]):
                    dlv = e["dlv"] if own else cdlv[j]
                    lanes[j] = advance(lanes[j], tau, inputs_of(rows, tau, dlv))
                if act[j] and tau >= cend[j]:
                    act[j] = False
    return lanes[0], ring


def session_calls(rows_remote, arrive, maxp, nc):
    rows2 = np.stack([np.zeros(nc, np.uint8), rows_remote], axis=1)
    out = o.p2p_sched_run(rows2, arrive, None, num_players=2, local_mask=1, max_prediction=maxp)
    assert out["rc"] == 0
    calls, cur, dlv = [], 0, -1
    for c in range(nc):
        dlv = max(dlv, int(arrive[c]))
        rb = int(out["rb_frame"][c])
        d = cur - rb if rb >= 0 else 0
        adv = int(out["advanced"][c])
        calls.append((cur, d, adv, dlv))
        cur += adv
    return calls


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    nc = int(sys.argv[2]) if len(sys.argv) > 2 else 160
    maxp = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    R = maxp + 1
    rng = np.random.default_rng(1)
    bad = 0
    for stalls in (False, True):
        arr = synth.jitter_arrivals(0, S, nc, maxp, stalls=stalls)
        rows = synth.gen_inputs(0, S, nc, 2, synth.MODEL_HELD)
        for s in range(S):
            calls = session_calls(rows[:, s, 1], arr[:, s], maxp, nc)
            seq_st, seq_ring = sequential(calls, rows[:, s, 1], R, None)
            # launches of random sizes, stages of random sizes
            st, ring, cur0, c = 0, {}, 0, 0
            while c < nc:
                n = int(rng.integers(1, 70))
                n = min(n, nc - c)
                stages, left = [], n
                while left:
                    k = min(left, int(rng.integers(1, 20)))
                    stages.append(k)
                    left -= k
                st, ring = time_aligned(calls[c:c + n] + calls[c + n:c + n + 1], rows[:, s, 1], R, maxp, stages,
                                        st, ring, cur0)
                c += n
                cur0 = calls[c][0] if c < nc else None
            ok = st == seq_st and ring == seq_ring
            bad += not ok
            if not ok and bad < 5:
                print("mismatch session", s, "stalls", stalls)
    print("sessions checked:", 2 * S, "mismatches:", bad)


if __name__ == "__main__":
    main()
