"""CPU check of nc_det.hip's run summation (k_det_runs + k_det_join): a Python model of
the sub-chunk run sums, the in-chunk join (the half-wave where a run starts adds the later
pieces in order) and the chunk-level join, run on 400 random run-length patterns (runs of
1-700 entries, invalid tails) against a plain segmented sum: every voxel written exactly
once, with its sum.

    python tools/det_join_sim.py
"""
import random

INV = -1  # the invalid key (out-of-grid corners, padding): sorted last, never written


def simulate(keys, vals, DSUB=16):
    """keys sorted (INV last), vals per entry -> {key: (sum, number of writes)}."""
    n = len(keys)
    DCH = 8 * DSUB
    out = {}

    def write(k, v):
        c = out.get(k, (0.0, 0))
        out[k] = (c[0] + v, c[1] + 1)

    nch = (n + DCH - 1) // DCH
    part = {}
    for b in range(nch):  # k_det_runs: one workgroup per chunk, half-wave hw per sub-chunk
        racc, rkey, rcnt, rnext, info = {}, {}, {}, {}, {}
        for hw in range(8):
            e0 = (b * 8 + hw) * DSUB
            cnt = 0 if e0 >= n else min(DSUB, n - e0)
            runs = []
            for i in range(cnt):
                k = keys[e0 + i]
                if runs and runs[-1][0] == k:
                    runs[-1][1] += vals[e0 + i]
                else:
                    runs.append([k, vals[e0 + i]])
            rkey[hw] = [r[0] for r in runs]
            racc[hw] = [r[1] for r in runs]
            rcnt[hw] = len(runs)
            nextk = keys[e0 + cnt] if (cnt > 0 and e0 + cnt < n) else INV
            prevk = keys[e0 - 1] if (0 < e0 <= n) else INV
            rnext[hw] = nextk if cnt > 0 else INV
            info[hw] = (cnt, prevk, nextk)
        for hw in range(8):
            cnt, prevk, nextk = info[hw]
            if cnt == 0:
                continue
            nr = rcnt[hw]
            kf, kl = rkey[hw][0], rkey[hw][nr - 1]
            cin = kf != INV and prevk == kf
            cout = kl != INV and nextk == kl
            if hw == 0 and cin:  # the run continuing from the previous chunk
                acc, open_, t = racc[0][0], nr == 1 and cout, 1
                while open_ and t < 8:
                    acc += racc[t][0]
                    open_ = rcnt[t] == 1 and rnext[t] == kf
                    t += 1
                part[(b, 0)] = acc
            closed = False
            if cout and not (nr == 1 and cin):  # the last run starts here and goes on
                acc, open_, t = racc[hw][nr - 1], True, hw + 1
                while open_ and t < 8:
                    acc += racc[t][0]
                    open_ = rcnt[t] == 1 and rnext[t] == kl
                    t += 1
                if open_:
                    part[(b, 0 if (hw == 0 and nr == 1) else 1)] = acc
                else:
                    racc[hw][nr - 1] = acc
                    closed = True
            for r in range(nr):
                k = rkey[hw][r]
                if k == INV or (r == 0 and cin) or (r == nr - 1 and cout and not closed):
                    continue
                write(k, racc[hw][r])
    for s in range(nch):  # k_det_join: runs crossing chunk boundaries, owned where they start
        e0, e1 = s * DCH, min(s * DCH + DCH, n)
        last, first = keys[e1 - 1], keys[e0]
        after = keys[e1] if e1 < n else keys[e1 - 1]
        before = keys[e0 - 1] if e0 > 0 else keys[e0]
        cont = last != INV and e1 < n and after == last
        single = first == last
        if not (cont and not (single and e0 > 0 and before == last)):
            continue
        acc, t = part[(s, 0 if single else 1)], s + 1
        while True:
            acc += part[(t, 0)]
            te = (t + 1) * DCH
            if te >= n or keys[te] != last:
                break
            t += 1
        write(last, acc)
    return out


def check(trials=400, seed=1):
    """Random run-length patterns against a plain segmented sum (see the module header)."""
    random.seed(seed)
    for trial in range(trials):
        n = random.randint(1, 3000)
        style = trial % 4
        keys = []
        k = 0
        while len(keys) < n:
            L = random.choice([1, 1, 2, 3, 5, 17, 40, 130, 300, 700]) if style else random.randint(1, 4)
            keys += [k] * L
            k += random.randint(1, 3)
        keys = keys[:n]
        if trial % 5 == 0:  # invalid tail (out-of-grid corners sort last)
            m = random.randint(0, n // 3)
            keys = keys[:n - m] + [INV] * m
        vals = [random.random() for _ in range(n)]
        out = simulate(keys, vals)
        ref = {}
        for kk, v in zip(keys, vals):
            if kk != INV:
                ref[kk] = ref.get(kk, 0.0) + v
        assert set(out) == set(ref), (trial, set(ref) ^ set(out))
        for kk in ref:
            assert out[kk][1] == 1, (trial, kk, out[kk])
            assert abs(out[kk][0] - ref[kk]) < 1e-9 * max(1, abs(ref[kk])), (trial, kk)


if __name__ == "__main__":
    check()
    print("ok")
