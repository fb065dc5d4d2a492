"""PCIe link use in a rocprofv3 --memory-copy-trace of the pipelined request stream: copies over
0.3 ms by direction, their mean duration, the fraction of the last N requests' span each
direction is busy, and the decode kernels' mean duration.
usage: python3 scripts/trace_links.py <dir with run_memory_copy_trace.csv> [N]"""
import collections
import csv
import os
import sys


def busy(iv):
    iv = sorted(iv)
    b, (cs, ce) = 0, iv[0][:2]
    for s, e, *_ in iv[1:]:
        if s > ce:
            b += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return b + ce - cs


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    rows = list(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))))
    ks = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"][12:]) for r in rows]
    by = collections.defaultdict(list)
    for c in cp:
        if c[1] - c[0] > 300_000:
            by[c[2]].append(c)
    h = sorted(by["HOST_TO_DEVICE"])[-n:]
    dd = sorted(by["DEVICE_TO_HOST"])[-n:]
    t0, t1 = min(h[0][0], dd[0][0]), max(h[-1][1], dd[-1][1])
    out = {"requests": n, "span_ms": round((t1 - t0) / 1e6, 2), "ms_per_request": round((t1 - t0) / 1e6 / n, 3),
           "h2d_ms_mean": round(sum(e - s for s, e, _ in h) / len(h) / 1e6, 3),
           "d2h_ms_mean": round(sum(e - s for s, e, _ in dd) / len(dd) / 1e6, 3),
           "h2d_busy": round(busy(h) / (t1 - t0), 3), "d2h_busy": round(busy(dd) / (t1 - t0), 3)}
    ev = sorted([(s, 1) for s, _, _ in dd] + [(e, -1) for _, e, _ in dd])
    c, last, hist = 0, ev[0][0], collections.Counter()
    for t, x in ev:
        hist[c] += t - last
        last, c = t, c + x
    tot = sum(hist.values())
    out["d2h_concurrency"] = {k: round(v / tot, 3) for k, v in sorted(hist.items())}
    kk = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"]) for k in ks]
    dec = [k for k in kk if k[0] >= t0 and ("wv_pcm" in k[2])]
    out["pcm_kernels"] = len(dec)
    out["pcm_kernel_ms_mean"] = round(sum(e - s for s, e, _ in dec) / max(1, len(dec)) / 1e6, 3)
    print(out)


if __name__ == "__main__":
    main()
