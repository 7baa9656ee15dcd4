"""Summarise KSS_STAMPS_FILE dumps (s_memrealtime, 100 MHz; one record per launch:
{kernel, shards} then the stamps).

k_schedule (shard 0, 8 stamps per pod): 0 pod start, 1 plan, 2 filter pass done, 3 filter
exchange done, 4 normalize pass done, 5 argmax exchange done, 6 commit + barrier done, 7 the
spread / inter-pod statistics and their exchange done (inside the filter phase).
k_simple (every shard, 16 per pod): 0 start, 1 pass B, 2 best-key reduction, 3 pass A,
4 statistics reduction (= publish), 5 exchange + barrier, 6 commit + ring store.  For
k_simple the arrival skew of the exchange is reported: per pod, the spread of the
shards' publish times, and the wait from the LAST publish to each shard's completion
(propagation + reductions).
k_spread (every shard, 16 per pod): 0 start, 1 stats pass, 2 stats exchange (E1) + minima,
3 filter pass, 4 filter exchange (E2), 5 PodTopologySpread score pass, 6 its exchange (E3),
7 normalize pass, 8 argmax exchange (E4), 9 commit + ring store.  Phases a pod skips
carry the previous stamp (duration 0)."""
import sys

import numpy as np

NAMES = ["plan", "filter", "x_filter", "normalize", "x_argmax", "commit"]
NAMES_SIMPLE = ["passB", "red_best", "passA", "red_stats", "xchg", "commit"]
NSTAMP_PODS = 256
NAMES_SPREAD = ["stats", "x_stats", "filter", "x_filter", "pts", "x_pts", "normalize", "x_argmax", "commit"]


def records(path):
    raw = np.fromfile(path, dtype=np.uint64)
    out, i = [], 0
    while i + 2 <= raw.size:
        kind, w = int(raw[i]), int(raw[i + 1])
        n = 8 * NSTAMP_PODS * (w if kind in (1, 2) else 1)
        out.append((kind, w, raw[i + 2:i + 2 + n].astype(np.int64)))
        i += 2 + n
    return out


def summarise(path):
    lines = []
    for kind, w, a in records(path):
        if kind == 0:
            a = a.reshape(-1, 8)
            a = a[(a[:, 0] > 0) & (a[:, 6] > 0)]
            d = np.diff(a[:, :7], axis=1) / 100.0
            tot = (a[:, 6] - a[:, 0]) / 100.0
            line = ("k_schedule " + " ".join(f"{n}={m:.2f}" for n, m in zip(NAMES, np.median(d, axis=0)))
                    + f" | pod={np.median(tot):.2f} us (n={len(a)})")
            if (a[:, 7] > 0).any():  # stamp 7: the statistics (+ their exchange) done inside `filter`
                st = (a[:, 7] - a[:, 1]) / 100.0
                line += f"\n  filter = statistics + exchange {np.median(st):.2f} + filter pass {np.median(d[:, 1] - st):.2f} us"
            lines.append(line)
            continue
        a = a.reshape(w, NSTAMP_PODS // 2, 16)
        if kind == 2:
            lines.append(spread_summary(w, a))
            if (a[0, :, 14] > 0).any():
                lines.append(spread_e2_detail(w, a))
            continue
        s0 = a[0]
        ok = (s0[:, 0] > 0) & (s0[:, 6] > 0)
        d = np.diff(s0[ok, :7], axis=1) / 100.0
        tot = (s0[ok, 6] - s0[ok, 0]) / 100.0
        line = (f"k_simple W={w} shard0: " + " ".join(f"{n}={m:.2f}" for n, m in zip(NAMES_SIMPLE, np.median(d, axis=0)))
                + f" | pod={np.median(tot):.2f} us (n={ok.sum()})")
        pub, done = a[:, :, 4], a[:, :, 5]
        good = (pub > 0).all(axis=0) & (done > 0).all(axis=0)
        if good.sum():
            p, dn = pub[:, good], done[:, good]
            last = p.max(axis=0)
            skew = (last - p.min(axis=0)) / 100.0
            after = (dn - last[None, :]) / 100.0
            late = np.bincount(p.argmax(axis=0), minlength=w)
            line += (f"\n  exchange: publish spread median {np.median(skew):.2f} us (p90 {np.percentile(skew, 90):.2f}),"
                     f" last publish -> done median {np.median(after):.2f} us (min {np.median(after.min(axis=0)):.2f}),"
                     f" latest shard most often {int(late.argmax())} ({late.max()}/{good.sum()} pods)")
            pa = (a[:, :, 3] - a[:, :, 0]) / 100.0
            line += f"\n  start -> passA done per shard: median {np.median(pa[:, good]):.2f} us, max over shards (median) {np.median(pa[:, good].max(axis=0)):.2f}"
        if ((s0[ok, 7] > 0) & (s0[ok, 8] > 0)).any():  # per-wave mode: statistics reduction detail
            q = s0[ok][(s0[ok, 7] > 0) & (s0[ok, 8] > 0)]
            seq = np.stack([q[:, 3], q[:, 7], q[:, 8], q[:, 4]], axis=1)
            dd = np.median(np.diff(seq, axis=1) / 100.0, axis=0)
            line += (f"\n  red_stats detail (shard 0): wave_red={dd[0]:.2f} write+barrier={dd[1]:.2f}"
                     f" combine={dd[2]:.2f} us")
        if (s0[ok, 14] > 0).any():  # window mode: exchange detail (slots 10-14)
            line += window_detail(s0[ok])
        lines.append(line)
    return "\n".join(lines)


def window_detail(s):
    """k_simple window exchange of shard 0: combine done (4) -> poll done (10) -> cut computed (11)
    -> [cut shard: rank scan done (12)] -> done (5); slot 14 = 1 + 2 (shard 0 holds the cut) + 4
    (the second exchange E2 was needed)."""
    f = s[:, 14]
    d1 = np.median((s[:, 10] - s[:, 4]) / 100.0)
    d2 = np.median((s[:, 11] - s[:, 10]) / 100.0)
    d3 = np.median((s[:, 5] - s[:, 11]) / 100.0)
    line = (f"\n  window (shard 0): publish+poll={d1:.2f} cut={d2:.2f} rest={d3:.2f} us;"
            f" shard 0 cut in {int(((f & 2) > 0).sum())}/{len(f)} pods, E2 needed in {int(((f & 4) > 0).sum())}")
    c = (f & 2) > 0
    if c.any():
        line += f"; as cut shard: rank scan {np.median((s[c, 12] - s[c, 11]) / 100.0):.2f} us"
    return line


def spread_summary(w, a):
    a = a[:, :, :10].copy()
    ok = (a[:, :, 0] > 0).all(axis=0) & (a[:, :, 9] > 0).all(axis=0)
    a = a[:, ok, :]
    for i in range(1, 9):  # skipped phases: duration 0
        z = a[:, :, i] == 0
        a[:, :, i][z] = a[:, :, i - 1][z]
    d = np.diff(a[0], axis=1) / 100.0
    tot = (a[0, :, 9] - a[0, :, 0]) / 100.0
    line = (f"k_spread W={w} shard0: " + " ".join(f"{n}={m:.2f}" for n, m in zip(NAMES_SPREAD, d.mean(axis=0)))
            + f" (means) | pod median {np.median(tot):.2f} us, mean {tot.mean():.2f} (n={ok.sum()})")
    for name, pub, done in (("E1", 1, 2), ("E2", 3, 4), ("E4", 7, 8)):
        p, dn = a[:, :, pub], a[:, :, done]
        used = (dn[0] > p[0])
        if not used.any():
            continue
        p, dn = p[:, used], dn[:, used]
        last = p.max(axis=0)
        skew = (last - p.min(axis=0)) / 100.0
        after = (dn - last[None, :]) / 100.0
        line += (f"\n  {name} ({used.sum()} pods): publish spread median {np.median(skew):.2f} us,"
                 f" last publish -> done median {np.median(after):.2f} us (min over shards {np.median(after.min(axis=0)):.2f})")
    return line


def spread_e2_detail(w, a):
    """E2 internals (slots 10-14 of shard 0): wave reduce + barrier, combine + barrier,
    publish, sweep done, fold + atomics (exchange return)."""
    s = a[0]
    ok = (s[:, 3] > 0) & (s[:, 14] > 0) & (s[:, 4] > 0)
    s = s[ok]
    seq = np.stack([s[:, 3], s[:, 10], s[:, 11], s[:, 12], s[:, 13], s[:, 14], s[:, 4]], axis=1)
    d = np.diff(seq, axis=1) / 100.0
    names = ["wave_red+bar", "combine+bar", "publish", "sweep", "fold+atomic", "bar+read"]
    return "  E2 detail (shard 0): " + " ".join(f"{n}={m:.2f}" for n, m in zip(names, np.median(d, axis=0)))


def latency_summary(path):
    """The first record of a stamps dump as a dict: kernel, shards, mean per-phase us of
    shard 0, and per exchange the median over pods of the fastest shard's wait from the last
    publish to completion (the exchange floor: propagation + combine)."""
    kind, w, a = records(path)[0]
    if kind == 0:
        a = a.reshape(-1, 8)
        a = a[(a[:, 0] > 0) & (a[:, 6] > 0)]
        d = np.diff(a[:, :7], axis=1) / 100.0
        return {"kernel": "k_schedule", "shards": w, "pods": int(len(a)),
                "phases_us": {n: float(m) for n, m in zip(NAMES, d.mean(axis=0))}}
    a = a.reshape(w, NSTAMP_PODS // 2, 16)
    if kind == 1:
        names, top, pairs = NAMES_SIMPLE, 6, (("exchange", 4, 5),)
        b = a[:, :, :7]
        ok = (b[:, :, 0] > 0).all(axis=0) & (b[:, :, 6] > 0).all(axis=0)
    else:
        names, top, pairs = NAMES_SPREAD, 9, (("stats", 1, 2), ("filter", 3, 4), ("argmax", 7, 8))
        b = a[:, :, :10].copy()
        ok = (b[:, :, 0] > 0).all(axis=0) & (b[:, :, 9] > 0).all(axis=0)
        for i in range(1, 9):
            z = b[:, :, i] == 0
            b[:, :, i][z] = b[:, :, i - 1][z]
    b = b[:, ok, :]
    if not ok.any():
        return {"kernel": "k_simple" if kind == 1 else "k_spread", "shards": w, "pods": 0}
    d = np.diff(b[0, :, :top + 1], axis=1) / 100.0
    out = {"kernel": "k_simple" if kind == 1 else "k_spread", "shards": w, "pods": int(ok.sum()),
           "phases_us": {n: round(float(m), 3) for n, m in zip(names, d.mean(axis=0))},
           "pod_us_shard0": round(float(((b[0, :, top] - b[0, :, 0]) / 100.0).mean()), 3), "exchange_floor_us": {}}
    for name, pub, done in pairs:
        p, dn = b[:, :, pub], b[:, :, done]
        used = dn[0] > p[0]
        if used.any():
            last = p[:, used].max(axis=0)
            out["exchange_floor_us"][name] = round(float(np.median((dn[:, used] - last[None, :]).min(axis=0)) / 100.0), 3)
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p, summarise(p))
