"""Summarise durable-log flush timelines (tools/dlog_bench DLOG_TIMELINE files; dev tool).

    python tools/dlog_timeline.py FILE...

Per file: the run's marks (appends started / returned / everything durable,
seconds since open), the flushes, the writer's busy time and its idle gaps
(from the first write's start to the last write's end), the time from a
segment's seal to its CRCs being patched in (the checksum's share of the
flush thread) and from there to its write starting, and what happened after
the last append returned (the drain: the last seal, checksum, write, sync).
"""
import sys

import numpy as np


def load(path):
    marks = {}
    rows = []
    for line in open(path):
        if line.startswith("# start"):
            p = line.split()
            marks = {p[i]: float(p[i + 1]) for i in range(1, len(p), 2)}
        elif not line.startswith("#") and line.strip():
            rows.append([float(x) for x in line.split()])
    return marks, np.array(rows)


def summary(path):
    m, r = load(path)
    sealed, ck, queued, ws, we, synced, nb = r.T
    busy = (we - ws).sum()
    span = we.max() - ws.min()
    gaps = ws[1:] - we[:-1]
    last = int(np.argmax(synced))
    return {
        "flushes": len(r), "MB_per_flush": nb.mean() / 1e6,
        "run_ms": (m["durable"] - m["start"]) * 1e3,
        "appended_ms": (m["appended"] - m["start"]) * 1e3,
        "first_write_ms": (ws.min() - m["start"]) * 1e3,
        "writer_busy_ms": busy * 1e3, "writer_span_ms": span * 1e3,
        "writer_idle_ms": (span - busy) * 1e3, "max_gap_ms": gaps.max() * 1e3 if len(gaps) else 0,
        "GBps_write": nb.sum() / busy / 1e9,
        "seal_to_checksummed_ms": np.median(ck - sealed) * 1e3,
        "checksummed_to_write_ms": np.median(ws - ck) * 1e3,
        "drain_ms": (m["durable"] - m["appended"]) * 1e3,
        "last_seal_after_appended_ms": (sealed[last] - m["appended"]) * 1e3,
        "last_write_ms": (we[last] - ws[last]) * 1e3,
    }


if __name__ == "__main__":
    for p in sys.argv[1:]:
        s = summary(p)
        print(p.split("/")[-1], " ".join(f"{k} {v:.2f}" if isinstance(v, float) else f"{k} {v}"
                                          for k, v in s.items()))
