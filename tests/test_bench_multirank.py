"""bench.py's N > 1 flow end to end, two ranks on the CPU (VERDICT r4 Next 5).

Each case launches `python -m torch.distributed.run --nproc-per-node 2`
(gloo, 127.0.0.1) on tests/_bench_rank.py, which runs bench.main() with the
engine replaced by a CPU stand-in whose RCCL all-gather is carried by gloo.
So the code that runs on the driver's 8-GPU node -- rendezvous, the timed
steps with their barrier and max-over-ranks, the ranks' identities, the
gather with rank 0's digest check, multi_rank_fields and the exit codes --
runs here unchanged, with only the collective and the kernels stubbed.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(mode: str, *extra: str, timeout: float = 240):
    env = dict(os.environ, STUB_MODE=mode, BENCH_GATHER_TIMEOUT_S="8", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(HERE, "_bench_rank.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--records-per-rank", "512", "--record-bytes", "256", "--no-cpu", "--no-pmc",
           "--sustain-seconds", "0", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r, lines


def check_line(rec):
    assert rec["n_gpus"] == 2 and rec["scaling"] == "weak"
    assert [r["rank"] for r in rec["ranks"]] == [0, 1]
    for r in rec["ranks"]:
        assert set(r) == {"rank", "device", "pci_bus_id", "launch_ms"}
    assert len(rec["digests"]) == 2
    # weak scaling: the whole job's bytes over the slowest rank's wall time
    assert rec["value"] > 0 and rec["config"]["global_batch"] == 2 * 512


def test_two_ranks_gather_verified():
    r, lines = run_ranks("ok")
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints the line
    rec = lines[0]
    check_line(rec)
    assert rec["distinct_gpus"] == 2 and rec["rccl_ranks"] == 2
    g = rec["gather"]
    assert g["verified"] is True and "error" not in g and g["bytes_per_rank"] == 512 * 4
    assert g["rccl_devices"] == [0, 1]


@pytest.mark.parametrize("mode", ["error", "short"])
def test_failed_or_short_gather_exits_4(mode):
    r, lines = run_ranks(mode)
    assert r.returncode != 0
    assert len(lines) == 1, r.stdout + r.stderr[-2000:]
    rec = lines[0]
    check_line(rec)
    assert rec["gather"].get("error"), rec["gather"]
    if mode == "short":
        assert rec["rccl_ranks"] == 1
    # torchrun reports the failing rank's exit code
    assert "exitcode  : 4" in r.stderr or "exit code 4" in r.stderr or "exitcode: 4" in r.stderr, \
        r.stderr[-2000:]


def test_ranks_on_one_gpu_exit_4_unless_rehearsal():
    r, lines = run_ranks("shared")
    assert r.returncode != 0 and len(lines) == 1
    assert lines[0]["distinct_gpus"] == 1 and lines[0]["gather"]["verified"] is True
    r, lines = run_ranks("shared", "--share-device")
    assert r.returncode == 0, r.stderr[-3000:]
    rec = lines[0]
    check_line(rec)
    assert rec["distinct_gpus"] == 1 and rec["gather"] is None and rec["rccl_ranks"] is None


def test_hung_collective_prints_the_line_then_exits_3():
    r, lines = run_ranks("hang")
    assert r.returncode != 0
    assert lines, r.stdout + r.stderr[-2000:]
    rec = lines[-1]
    check_line(rec)
    assert "timed out" in rec["gather"]["error"]
    assert "RCCL gather timed out" in r.stderr
