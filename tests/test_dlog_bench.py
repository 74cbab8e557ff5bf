"""The durable-log bench driver's modes on the CPU (tools/dlog_bench, built by
consus_amd/csrc/Makefile; bench.py's `durable_log` leg runs it on the GPU box).

Without a GPU the log's batches complete on the engine's counted CPU path, so
every mode runs here: the writes dropped (DLOG_SINK, the leg's third
workload), pinned staging arenas forced (DLOG_PINNED, every engine of the leg),
the per-flush timeline (DLOG_TIMELINE, tools/dlog_timeline.py), and the
reference scheme (REF_SCHEME: every appender checksums its own frame with the
reference crc32c.cc, txman/durable_log.cc:215-218) with configs[2]'s entry
lengths.  Each run replays the log byte-exact (except the sink, which keeps
nothing) and prints one JSON line.
"""
import json
import os
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
BENCH = os.path.join(REPO, "tools", "dlog_bench")
REF = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")


def run(env_extra, threads=3, per=1500, tmp=None):
    d = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        env = dict(os.environ, **env_extra)
        r = subprocess.run([BENCH, os.path.join(d, "log"), str(threads), str(per), "42", "1024"],
                           capture_output=True, text=True, timeout=180, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
        files = {f: os.path.getsize(os.path.join(d, "log", f)) for f in ("file_a", "file_b")}
        return out, files
    finally:
        shutil.rmtree(d, ignore_errors=True)


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(BENCH):
        pytest.skip("tools/dlog_bench not built (python -c 'import __graft_entry__ as g; g.build()')")


def test_sink_drops_the_writes():
    out, files = run({"FAKE_CRC": "1", "DLOG_SINK": "1"})
    assert out["sink"] is True and not out.get("error")
    assert out["appends"] == 4500 and out["replayed"] == 4500 and out["replay_bad"] == 0
    assert files == {"file_a": 0, "file_b": 0}


def test_pinned_arenas_and_timeline():
    with tempfile.NamedTemporaryFile(suffix=".txt", delete=False) as f:
        tl = f.name
    try:
        out, files = run({"DLOG_PINNED": "1", "DLOG_TIMELINE": tl})
        assert out["sink"] is False and not out.get("error")
        assert out["replayed"] == out["appends"] == 4500 and out["replay_bad"] == 0
        assert sum(files.values()) == out["frame_bytes"]
        rows = [list(map(float, x.split())) for x in open(tl) if x.strip() and not x.startswith("#")]
        assert 1 <= len(rows) <= out["flushes"] + 1
        for r in rows:
            # sealed <= checksummed <= queued <= write start <= write end <= synced, bytes > 0
            assert len(r) == 7 and all(a <= b + 1e-9 for a, b in zip(r[:6], r[1:6])) and r[6] > 0
        assert sum(r[6] for r in rows) == out["frame_bytes"]
    finally:
        os.unlink(tl)


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built")
def test_reference_scheme_with_zipf_entries():
    out, files = run({"REF_CRC_SO": REF, "REF_SCHEME": "1", "DLOG_ENTRY": "zipf"}, per=400)
    assert out["engine"] == "reference-scheme" and "zipf" in out["entries"]
    assert out["replayed"] == out["appends"] == 1200 and out["replay_bad"] == 0
    assert sum(files.values()) == out["frame_bytes"]
