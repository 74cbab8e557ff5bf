#!/usr/bin/env python3
"""bench.py -- device-resident CRC-32C throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--records-per-rank R]

A "step" is one pass of the hot path -- consus::crc32c over every record of
one batch (common/crc32c.cc:122-126, the per-record call of
txman/durable_log.cc:215-218) -- done by the HIP kernels through the C ABI
(include/consus_crc32c.h, mi_crc32c_batch_fixed with MI_CRC32C_DEVICE).

Workload (N=1): BASELINE.json configs[1] -- 1M x 4 KiB records resident in
HBM, bytes = splitmix64 stream of seed 0xC0DE, generated on
the device before timing.  N>1 (torchrun, one process per GPU): every rank
owns its own 2M-record shard of the same global stream (record offset
rank*R; N = 8 is configs[3], 16M x 4 KiB), so per-GPU work is fixed
("scaling": "weak") and no collective runs inside the timed region (records
are independent).  After
timing, every rank's CRC vector is reduced on its GPU to a digest; the
digests are compared with the committed golden values (tests/golden).

The JSON line also carries
  roofline      algorithmic bytes per launch (sum of record lengths) / the
                launch's average duration from HIP events on the engine's
                stream, against the MI355X HBM3E peak (8 TB/s); `traffic` =
                2 x FETCH_SIZE from a separate rocprofv3 --pmc pass (gfx950
                reports half of wide streaming reads, MI355X_MICROARCH.md HBM)
  cpu_baseline  the reference common/crc32c.cc itself (oracle/_ref, compiled
                unmodified) on the host cores, over a bounded sample of the
                same records (rank 0, N=1 only): its dispatched path on every
                CPU this process may use (min of affinity and cgroup quota,
                both reported with nproc and the model), a 1/4/16/all-thread
                sweep, and its slicing-by-8 path once

Other workloads (--config, one JSON line each; see --help): zipf
(configs[2]; at N > 1 sharded by bytes across the GPUs), single (one 4 GiB device record; at N > 1 one record split
across the GPUs), stream (configs[4], host segments through the H2D/CRC/D2H
pipeline), pcie4k (configs[1] bytes starting in pinned host memory), dlog
(durable-log appends/s).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

_T0 = time.perf_counter()


def progress(msg: str) -> None:
    """One line per stage on stderr (stdout carries only the JSON line): a
    long default run shows where it is."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GiB/s CRC32C over device-resident 4 KiB records; % of HBM read peak"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E datasheet peak (MI355X_MICROARCH.md)
SEED = 0xC0DE
RECORD = 4096
KERNEL_NAME = "crc32c_fixed_pipe_kernel"  # 4 KiB records: G = 4 groups, no inits
KERNEL_MATCH = "crc32c_fixed"             # PMC rows: either fixed-length kernel


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 200 for the device-resident configs -- a "
                         "0.13-0.17 s timed region, so a short clock or power transient moves "
                         "the line by a fraction of a percent; 50 for stream/pcie4k/dlog)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps before the K timed ones (default 300 for the "
                         "device-resident configs -- about 0.2 s, the clock ramp: with 5 the "
                         "timed launches ran 1-2.5 %% below the sustained rate -- and 5 for "
                         "stream/pcie4k/dlog)")
    ap.add_argument("--sustain-seconds", type=float, default=8.0,
                    help="fixed4k: after the timed region, launch back to back for this long and "
                         "report the sustained per-GPU rate (clock/power droop check; it also keeps "
                         "the GPU busy long enough for an external utilisation sampler; 0 = off)")
    ap.add_argument("--config", default="fixed4k",
                    choices=["fixed4k", "zipf", "stream", "pcie4k", "single", "dlog"],
                    help="fixed4k = BASELINE configs[1] (headline, default); zipf = configs[2] "
                         "(at N > 1 its stream continued to N x 1M records, sharded by bytes); "
                         "stream = configs[4] (64 MiB host segments, H2D+CRC+D2H); pcie4k = "
                         "configs[1] bytes starting in pinned host memory; single = the same "
                         "4 GiB as ONE device-resident record (long-record path, SURVEY 8(f)4; "
                         "at N > 1 one N x 4 GiB record split across the GPUs, SURVEY 8(e)); "
                         "dlog = the durable-log front-end (SURVEY 8(f)1): appends/s of 8 "
                         "threads, GPU batch CRC per flushed segment")
    ap.add_argument("--segments", type=int, default=None,
                    help="stream/pcie4k: 64 MiB segments per step (default 16 for stream; 64 for "
                         "pcie4k = the whole 1M-record configs[1] batch, checked against its "
                         "golden block digest)")
    ap.add_argument("--records-per-rank", type=int, default=None,
                    help="default: 1M (configs[1]) on one GPU, 2M per GPU when N > 1, so that "
                         "N = 8 is configs[3] (16M x 4 KiB across 8 GPUs)")
    ap.add_argument("--record-bytes", type=int, default=RECORD)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="wall budget of each CPU-baseline leg (single, all-threads)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-legs", action="store_true",
                    help="fixed4k at N = 1: skip the other single-GPU BASELINE configs that the "
                         "headline line carries by default (configs[2] zipf, configs[4] stream, "
                         "the PCIe-inclusive configs[1] rate)")
    ap.add_argument("--leg-sustain-seconds", type=float, default=2.0,
                    help="zipf: back-to-back steps after the timed region for this long (0 = off)")
    ap.add_argument("--leg-cpu-seconds", type=float, default=3.0,
                    help="zipf/stream/pcie4k: wall budget of the reference-CPU leg on the same "
                         "bytes")
    ap.add_argument("--child-pmc", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the RCCL all-gather of the CRC vectors after the timed region")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank uses device 0 (no RCCL gather)")
    args = ap.parse_args()
    if args.warmup is None:
        args.warmup = 300 if args.config in ("fixed4k", "zipf", "single") else 5
    if args.steps is None:
        args.steps = 200 if args.config in ("fixed4k", "zipf", "single") else 50
    return args


def golden_digests():
    p = os.path.join(REPO, "tests", "golden", "digests.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


# ---- HBM traffic from a separate rocprofv3 --pmc pass ---------------------------
def pmc_traffic(args) -> tuple[float | None, str]:
    """Run this script under `rocprofv3 --pmc FETCH_SIZE` (its own pass, no
    tracing domains) and return corrected HBM read bytes per launch of the
    fixed kernel (fixed4k) or per step of the variable path (zipf: every
    cost/hash (sorted path) or plan, chunk and finalize (piece path)
    dispatch of one step; stream/pcie4k: every CRC kernel of one step's
    segments -- the H2D/D2H copies are DMA, not kernels)."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    out = tempfile.mkdtemp(prefix="pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [exe, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", out, "-o", "pmc",
           "--", sys.executable, os.path.abspath(__file__), "--child-pmc",
           "--config", args.config,
           "--records-per-rank", str(args.records_per_rank),
           "--record-bytes", str(args.record_bytes)]
    try:
        subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, cwd=out)
    except Exception as e:  # noqa: BLE001 -- traffic is optional, the bench is not
        return None, f"rocprofv3 pass failed: {e}"
    fixed = args.config in ("fixed4k", "single")  # single: the same code on its 4 KiB chunks
    step_kernels = ("sorted_cost_kernel", "crc32c_sorted_kernel",  # the sorted path
                    "plan_", "long_items", "crc32c_chunk_kernel", "crc32c_finalize", "long_finalize",
                    "crc32c_direct_kernel")
    vals = []
    for path in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if row.get("Counter_Name") != "FETCH_SIZE":
                    continue
                match = "crc32c_span_chunk" if args.config == "single" else KERNEL_MATCH
                if (fixed and match in name) or \
                        (not fixed and any(k in name for k in step_kernels)):
                    vals.append(float(row["Counter_Value"]))
    shutil.rmtree(out, ignore_errors=True)
    if not vals:
        return None, "no FETCH_SIZE rows for the kernel"
    # FETCH_SIZE is in KiB; gfx950 tallies 128-B requests of wide streaming
    # reads at 64 B, so double it (MI355X_MICROARCH.md, HBM).
    if fixed:
        return 2.0 * 1024.0 * float(np.median(vals)), \
            f"{len(vals)} dispatches, median, x2 gfx950 correction"
    steps = PMC_CHILD_STEPS if args.config == "zipf" else 1
    return 2.0 * 1024.0 * sum(vals) / steps, \
        f"sum over the step's {len(vals) // steps} kernel dispatches ({steps} steps), x2 gfx950 " \
        f"correction"


PMC_CHILD_STEPS = 3


def sub_args(args, config: str, **kw):
    """A copy of the command's arguments for another workload (bench legs)."""
    s = argparse.Namespace(**vars(args))
    s.config = config
    s.records_per_rank = 1 << 20
    s.segments = None
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def usable_cpus() -> tuple[int, dict]:
    cpus = host_cpus()
    usable = cpus["affinity"]
    if cpus["cgroup_quota_cpus"]:
        usable = max(1, min(usable, int(cpus["cgroup_quota_cpus"])))
    return usable, cpus


def timed_rate(fn, nbytes: int, seconds: float) -> tuple[float, int]:
    """GiB/s of fn() over nbytes, repeated for about `seconds` after one warm call."""
    fn()
    passes, t0 = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return passes * nbytes / dt / 2**30, passes


# ---- N > 1: the optional RCCL gather (BASELINE configs[3]) -----
def rccl_gather(E, dist, rank: int, world: int, out, R: int, digests, rec) -> dict:
    """All-gather every rank's CRC vector over RCCL (xGMI), outside the timed
    region; rank 0 checks each gathered block against the rank's own digest.
    A watchdog ends every rank if RCCL never returns; rank 0 first prints its
    bench line (`rec`) with the gather marked as timed out, then every rank
    exits 3, so the launcher sees the hung collective (the bench line above
    it stays valid: the gather is outside the timed region)."""
    import threading
    done = threading.Event()
    # BENCH_GATHER_TIMEOUT_S: the watchdog's limit (tests/test_bench_multirank.py
    # drives the hung-collective exit with a short one)
    limit = float(os.environ.get("BENCH_GATHER_TIMEOUT_S", "120"))

    def watchdog():
        if not done.wait(limit):
            if rec is not None:
                rec["gather"] = {"collective": "rccl all-gather", "error": f"timed out after {limit:g} s"}
                print(json.dumps(rec), flush=True)
            print(f"rank {rank}: RCCL gather timed out after {limit:g} s", file=sys.stderr, flush=True)
            os._exit(3)
    threading.Thread(target=watchdog, daemon=True).start()
    try:
        uid = [E.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        E.comm_init(uid[0], world, rank)
        info = E.comm_info()  # RCCL's own count of ranks and this rank's device
        views = [None] * world
        dist.all_gather_object(views, info)
        recv = E.DeviceBuffer(world * R * 4)
        E.comm_allgather_u32(out, R, recv)            # warm-up: connection setup
        times = []
        for _ in range(5):
            dist.barrier()
            t0 = time.perf_counter()
            E.comm_allgather_u32(out, R, recv)        # synchronous on the engine stream
            times.append(time.perf_counter() - t0)
        ok = all(E.crc32c_device(recv, R * 4, offset=i * R * 4) == digests[i]
                 for i in range(world)) if rank == 0 else None
        E.comm_destroy()
        res = {"collective": "rccl all-gather of u32 CRC vectors", "bytes_per_rank": R * 4,
               "ms_median": round(1e3 * float(np.median(times)), 4), "verified": ok,
               "rccl_ranks": info["nranks"],
               "rccl_devices": [v["device"] for v in views]}
        if rank == 0 and (ok is not True or info["nranks"] != world):
            res["error"] = f"gather check failed: verified={ok}, rccl_ranks={info['nranks']}"
    except Exception as e:  # noqa: BLE001 -- the gather is optional, the bench line is not
        res = {"collective": "rccl all-gather", "error": str(e)[:200]}
    done.set()
    return res


def multi_rank_fields(rec: dict, ranks: list, gather, world: int, share_device: bool) -> int:
    """The N > 1 keys of the bench line: every rank's identity (rank, HIP
    device, PCI bus id, per-launch ms), the count of distinct GPUs, the RCCL
    gather's result and its communicator's rank count.  Returns the exit code:
    4 when the gather failed or did not verify, or when the ranks did not land
    on `world` distinct GPUs (outside a one-GPU rehearsal) -- the line says
    what, the exit code makes it fail (tests/test_bench_shape.py)."""
    rec["ranks"] = ranks
    rec["distinct_gpus"] = len({r["pci_bus_id"] for r in ranks})
    rec["gather"] = gather
    rec["rccl_ranks"] = gather.get("rccl_ranks") if gather else None
    bad = bool((gather or {}).get("error")) or (gather is not None and rec["rccl_ranks"] != world) \
        or (not share_device and rec["distinct_gpus"] != world)
    return 4 if bad else 0


def rank_identity(E, dist, rank: int, device: int, launch_ms: float) -> list | None:
    """Every rank's (rank, HIP device, PCI bus id, per-launch ms), gathered on
    the gloo control plane: the line shows which physical GPUs ran."""
    try:
        pci = E.device_pci_bus_id(device)
    except Exception as e:  # noqa: BLE001
        pci = f"unknown ({e})"[:60]
    me = {"rank": rank, "device": device, "pci_bus_id": pci, "launch_ms": round(launch_ms, 4)}
    if dist is None:
        return [me]
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, me)
    return allr


# ---- CPU baseline: the reference itself ---------------------------------------
def host_cpus() -> dict:
    """What this process may run on: the machine's CPUs (nproc), this
    process's affinity mask, the cgroup CPU quota (cpu.max), and the model."""
    info = {"nproc": os.cpu_count() or 1,
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
            else os.cpu_count() or 1,
            "cgroup_quota_cpus": None, "model": ""}
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and parts and parts[0] != "max":
            info["cgroup_quota_cpus"] = round(int(parts[0]) / int(parts[1]), 2)
        elif path.endswith("quota_us") and parts and int(parts[0]) > 0:
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    info["cgroup_quota_cpus"] = round(int(parts[0]) / int(f.read()), 2)
            except OSError:
                pass
        break
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return info


def cpu_baseline(args) -> dict:
    """The reference common/crc32c.cc itself (oracle/_ref, compiled unmodified)
    over a bounded sample of the same records, on every CPU this process may
    use: threads = min(affinity, cgroup quota) -- nothing is capped by a
    constant.  A 1 / 4 / 16 / all-thread sweep goes with it."""
    from oracle.oracle import Oracle, Reference, reference_available
    cpus = host_cpus()
    if not reference_available():
        return {"value": None, "unit": "GiB/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/libref_crc32c.so not built", "host": cpus}
    ref, orc = Reference(), Oracle()
    L = args.record_bytes
    # 1 GiB sample of the same records: 4x the 256 MB L3 of the EPYC hosts, so
    # the CPU streams from DRAM as the GPU streams from HBM
    n = (1 << 30) // L
    buf = orc.fill(n * L, SEED, 0)
    usable = cpus["affinity"]
    if cpus["cgroup_quota_cpus"]:
        usable = max(1, min(usable, int(cpus["cgroup_quota_cpus"])))

    def rate(th, seconds):
        ref.fixed(buf, L, L, n, threads=th)  # warm: thread start-up, caches, clocks
        passes, t0 = 0, time.perf_counter()
        while True:
            ref.fixed(buf, L, L, n, threads=th)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                return passes * n * L / dt / 2**30, passes
    crc_ref = ref.fixed(buf, L, L, 64, threads=1)
    leg = args.cpu_seconds / 2
    sweep = {}
    for th in sorted({1, 4, 16, usable} | ({cpus["affinity"]} if cpus["affinity"] <= 256 else set())):
        if th > cpus["affinity"]:
            continue
        sweep[str(th)] = round(rate(th, leg)[0], 2)
    multi, pm = rate(usable, args.cpu_seconds)
    single = sweep["1"]
    # the reference's other path, slicing-by-8 (common/crc32c.cc:40-48, 594-634;
    # taken on CPUs without SSE4.2), once over 256 MiB of the sample
    t0 = time.perf_counter()
    ref.crc32c(0, buf, 256 << 20, impl="sw")
    sb8 = (256 << 20) / (time.perf_counter() - t0) / 2**30
    return {"value": round(multi, 2), "unit": "GiB/s", "cores": usable, "kind": "reference",
            "single_thread_value": single,
            "slicing_by_8_single_thread_value": round(sb8, 2),
            "thread_sweep_gib_s": sweep,
            "host": cpus,
            "sample": f"first {n} x {L} B of the same records ({n * L >> 20} MiB, host DRAM); "
                      f"common/crc32c.cc compiled unmodified, "
                      f"{'sse42 crc32q' if ref.lib.ref_dispatch_is_sse42() else 'slicing-by-8'}; "
                      f"{pm} passes x {usable} std::threads = min(affinity {cpus['affinity']}, "
                      f"cgroup quota {cpus['cgroup_quota_cpus']}), nproc {cpus['nproc']}; "
                      f"{cpus['model']}",
            "first_crc": int(crc_ref[0])}


def _interp(points, n):
    """Linear interpolation of {bytes: us} at n bytes (clamped to the ends)."""
    pts = sorted((int(k), float(v)) for k, v in points.items())
    if not pts:
        return None
    if n <= pts[0][0]:
        return pts[0][1] * n / pts[0][0]
    for (n0, t0), (n1, t1) in zip(pts, pts[1:]):
        if n <= n1:
            return t0 + (t1 - t0) * (n - n0) / (n1 - n0)
    (n0, t0), (n1, t1) = pts[-2], pts[-1]
    return t1 + (t1 - t0) * (n - n1) / (n1 - n0)


def run_dlog(args, compact: bool = False) -> dict:
    """The batching durable log driven as txman drives it (tools/dlog_bench.cc):
    8 threads append concurrently, the caller waits for the watermark to cover
    every record, then the log is replayed (GPU-verified scan of both segment
    files) and every record checked byte-exact.  Segment files on tmpfs
    (/dev/shm): fsync is free there, so this is the front-end and checksum
    rate, not a disk's.  Two entry-length workloads: uniform 42-1024 B, and
    configs[2]'s Zipf 64 B - 64 KiB (where one core's crc32q is a real cost).
    Four engines, runs interleaved (>= 7 each), median and IQR reported:
      gpu               the batching front-end, one GPU batch per flushed
                        segment (flushes below the measured GPU/CPU crossover
                        on the flush thread's CPU path, counted);
      reference-scheme  the reference's own placement (txman/durable_log.cc:
                        215-218): every appender computes its frame's CRC with
                        common/crc32c.cc (oracle/_ref, compiled unmodified) on
                        its own thread -- the CPU baseline of this line;
      reference-cpu     the same reference function on the flush thread;
      no-checksum       a no-op flush checksum: the front-end's own ceiling."""
    exe = os.path.join(REPO, "tools", "dlog_bench")
    d = tempfile.mkdtemp(prefix="dlog_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    threads = 8
    from oracle.oracle import REF_SO, reference_available
    workloads = [("uniform", {"per": 400_000, "lo": 42, "hi": 1024, "env": {},
                              "what": "entry lengths uniform 42-1024 B; segment files on tmpfs"}),
                 ("zipf", {"per": 25_000, "lo": 0, "hi": 0, "env": {"DLOG_ENTRY": "zipf"},
                           "what": "entry lengths of configs[2]: Zipf 64 B - 64 KiB; segment files "
                                   "on tmpfs"}),
                 # round 6: storage faster than the front-end (the writer's pwrite and
                 # the fsync skipped): the log's rate is its appenders' and its
                 # checksum's, which is where the checksum's placement shows
                 ("zipf_sink", {"per": 25_000, "lo": 0, "hi": 0,
                                "env": {"DLOG_ENTRY": "zipf", "DLOG_SINK": "1"},
                                "what": "entry lengths of configs[2]; storage faster than the "
                                        "front-end (pwrite and fsync skipped, no replay)"})]
    # every engine stages frames in the same pinned arenas (round 6: with
    # ordinary memory the CPU engines' appenders page-faulted their arenas and
    # flushed smaller segments, a different log configuration)
    engines = [("gpu", {})]
    if reference_available() and not args.no_cpu:
        engines.append(("reference-scheme", {"REF_CRC_SO": REF_SO, "REF_SCHEME": "1", "DLOG_PINNED": "1"}))
        engines.append(("reference-cpu", {"REF_CRC_SO": REF_SO, "DLOG_PINNED": "1"}))
    engines.append(("no-checksum", {"FAKE_CRC": "1", "DLOG_PINNED": "1"}))
    nruns = max(7, args.steps // 4)
    # BENCH_DLOG_SCALE: fewer appends per run (CPU rehearsals of this leg only)
    scale = float(os.environ.get("BENCH_DLOG_SCALE", "1"))
    for _, w in workloads:
        w["per"] = max(100, int(w["per"] * scale))
    runs = {w: {e: [] for e, _ in engines} for w, _ in workloads}
    try:
        for i in range(nruns):
            for wname, w in workloads:
                if i == 0:  # one progress line per workload (the runs are interleaved)
                    progress(f"durable log: {wname}, {nruns} interleaved runs x {len(engines)} engines")
                for name, extra in engines:
                    env = dict(os.environ)
                    env.update(w["env"])
                    env.update(extra)
                    if runs[wname][name] or wname != workloads[0][0]:
                        env["DLOG_NO_PROBES"] = "1"  # the GPU engine's one-off probes: first run only
                    r = subprocess.run([exe, os.path.join(d, "log"), str(threads), str(w["per"]),
                                        str(w["lo"]), str(w["hi"])],
                                       capture_output=True, text=True, timeout=300, env=env)
                    if r.returncode != 0:
                        raise RuntimeError(f"dlog_bench ({wname}/{name}) failed: "
                                           f"{r.stdout[-500:]} {r.stderr[-500:]}")
                    runs[wname][name].append(json.loads(r.stdout.strip().splitlines()[-1]))
                    shutil.rmtree(os.path.join(d, "log"), ignore_errors=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)

    def q(xs, p):
        return float(np.percentile(np.asarray(xs, dtype=float), p))

    def median_run(rs):
        return sorted(rs, key=lambda x: x["appends_per_s"])[(len(rs) - 1) // 2]  # (lower) median

    def per_flush(x):
        f = max(x["flushes"], 1)
        return {"flushes": x["flushes"], "host_flushes": x.get("host_flushes", 0),
                "frame_bytes_per_flush": round(x["frame_bytes"] / f),
                "us_per_flush": {k: round(v / f * 1e6, 2) for k, v in x["flush_s"].items()},
                "checksum_s": round(x["flush_s"]["batch_crc"], 4), "run_s": round(x["durable_s"], 4)}

    def summary(rs):
        ap = [x["appends_per_s"] for x in rs]
        gb = [x["frame_GiB_per_s"] for x in rs]
        return {"appends_per_s": {"median": round(q(ap, 50), 1), "q1": round(q(ap, 25), 1),
                                  "q3": round(q(ap, 75), 1)},
                "frame_gib_per_s": {"median": round(q(gb, 50), 4), "q1": round(q(gb, 25), 4),
                                    "q3": round(q(gb, 75), 4)},
                "durable_latency_us": {
                    "p50_median": round(q([x["durable_latency_us"]["p50"] for x in rs], 50), 1),
                    "p99_median": round(q([x["durable_latency_us"]["p99"] for x in rs], 50), 1)},
                "runs": [round(v, 1) for v in ap]}

    def versus(a, b):
        """a against b: ratio of medians, and whether the IQRs separate."""
        sa, sb = a["appends_per_s"], b["appends_per_s"]
        verdict = ("higher" if sa["q1"] > sb["q3"] else "lower" if sa["q3"] < sb["q1"]
                   else "within run spread")
        ga, gb = a["frame_gib_per_s"], b["frame_gib_per_s"]
        return {"appends_ratio": round(sa["median"] / max(sb["median"], 1e-9), 3),
                "gib_ratio": round(ga["median"] / max(gb["median"], 1e-9), 3),
                "beyond_spread": verdict}

    out = {}
    for wname, w in workloads:
        eng = {name: summary(runs[wname][name]) for name, _ in engines}
        res = {"workload": f"{threads} threads x {w['per']} appends, {w['what']}; then wait for "
                           f"the watermark", "engines": eng}
        res["gpu_vs"] = {name: versus(eng["gpu"], eng[name]) for name, _ in engines if name != "gpu"}
        best = dict(median_run(runs[wname]["gpu"]))
        first = runs[workloads[0][0]]["gpu"][0]  # the one run that took the engine's probes
        for k in ("empty_batch_us", "cpu_batch_us", "link_us"):
            best[k] = first.get(k, best.get(k))
        pf = per_flush(best)
        # The per-flush bound: the cheaper of the two routes the log chooses
        # between by size (durable_log.cc host_batch_max).  The GPU batch's:
        # its floor (a one-frame round trip through the log's entry point,
        # measured by dlog_bench) plus the bytes at the host link's ~55 GB/s.
        # The flush thread's CPU: the reference crc32c.cc engine's own time
        # per byte on the flush thread in the same job (the same frames, just
        # written by the appenders on other cores), at this flush's size.  The
        # CPU loop on a warm buffer (cpu_batch_us_at_flush, dlog_bench) is
        # reported beside it: flushed frames are not in this core's cache.
        nb = pf["frame_bytes_per_flush"]
        gpu_bound = best.get("empty_batch_us", 0.0) + nb / 55e3
        cpu_us = _interp(best.get("cpu_batch_us", {}), nb)
        ref_us = None
        if "reference-cpu" in runs[wname]:
            rc = per_flush(median_run(runs[wname]["reference-cpu"]))
            pf["reference_cpu_us_per_flush"] = rc["us_per_flush"]["batch_crc"]
            pf["reference_cpu_frame_bytes_per_flush"] = rc["frame_bytes_per_flush"]
            if rc["frame_bytes_per_flush"]:
                ref_us = rc["us_per_flush"]["batch_crc"] * nb / rc["frame_bytes_per_flush"]
        bound = min(gpu_bound, ref_us) if ref_us else gpu_bound
        pf.update({"empty_batch_us": best.get("empty_batch_us", 0.0),
                   "gpu_batch_bound_us": round(gpu_bound, 2),
                   "reference_cpu_us_at_flush": None if ref_us is None else round(ref_us, 2),
                   "cpu_batch_us_at_flush": None if cpu_us is None else round(cpu_us, 2),
                   "batch_crc_bound_us": round(bound, 2),
                   "batch_crc_vs_bound": round(pf["us_per_flush"]["batch_crc"] / bound, 3),
                   "routed_to_cpu": f"{pf['host_flushes']} of {pf['flushes']} flushes"})
        res["flush"] = pf
        if not compact:
            res["runs_detail"] = runs[wname]
        out[wname] = res
    uni = out["uniform"]["engines"]
    cpu = None
    if "reference-scheme" in uni:
        rs = uni["reference-scheme"]
        cpu = {"value": rs["appends_per_s"]["median"], "unit": "appends/s", "cores": threads,
               "kind": "reference",
               "sample": "the same front-end, appenders and entries (uniform 42-1024 B), with each "
                         "appender computing its frame's CRC by the reference common/crc32c.cc "
                         "(oracle/_ref, compiled unmodified; crc32q dispatch) on its own thread, "
                         "as txman/durable_log.cc:215-218 does; median of the interleaved runs"}
    return {"metric": "durable-log appends/s, 8 appending threads, GPU batch CRC per flushed "
                      "segment (txman/durable_log.cc append contract)",
            "value": uni["gpu"]["appends_per_s"]["median"], "unit": "appends/s", "n_gpus": 1,
            "steps": nruns, "warmup": 0,
            "ms_per_step": round(median_run(runs["uniform"]["gpu"])["durable_s"] * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: splitmix64 entry bytes; uniform 42-1024 B and Zipf 64 B-64 KiB lengths",
            "config": {"workload": "8 appending threads; uniform and Zipf entries on tmpfs, Zipf "
                                   "entries on a sink faster than the front-end; "
                                   f"{nruns} interleaved runs per engine and workload"},
            "workloads": out, "roofline": None, "cpu_baseline": cpu,
            "digest_verified": all(x["replayed"] == x["appends"] and x["replay_bad"] == 0
                                   for wn, w in runs.items() for name, rs in w.items()
                                   if name != "no-checksum" and not wn.endswith("_sink")
                                   for x in rs)}


def run_secondary(args, E, traffic=(None, "skipped")) -> dict:
    """Configs 3 and 5 and the host-inclusive rate of config 2 (one GPU)."""
    from consus_amd import workload as W
    gold = golden_digests()
    res = {"n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u32", "cpu_baseline": None}
    if args.config == "zipf":
        R = args.records_per_rank
        off, ln, total = W.zipf_records(R)
        data = E.DeviceBuffer(total + 16)
        data.fill_splitmix64(W.DATA_SEED)
        d_off, d_len, out = E.DeviceBuffer(R * 8), E.DeviceBuffer(R * 4), E.DeviceBuffer(R * 4)
        d_off.upload(off)
        d_len.upload(ln)
        if args.child_pmc:
            for _ in range(PMC_CHILD_STEPS):
                E.device_batch(data, d_off, d_len, R, out, total_bytes=total)
            return {}
        # one synchronous step (it checks the size hint's overflow flag), then
        # the warm-up back to back, as the timed steps run
        E.device_batch(data, d_off, d_len, R, out, total_bytes=total)
        for _ in range(args.warmup):
            E.device_batch(data, d_off, d_len, R, out, total_bytes=total, asynchronous=True)
        E.sync()
        sorted0 = E.stats().get("sorted_batches", 0)
        t0 = time.perf_counter()
        E.timer_start()
        for _ in range(args.steps):
            E.device_batch(data, d_off, d_len, R, out, total_bytes=total, asynchronous=True)
        ev = E.timer_stop() / args.steps
        wall = (time.perf_counter() - t0) / args.steps
        dig = E.crc32c_device(out, R * 4)
        g = gold.get("zipf_seed0x5eed_data0xda7a5eed_1048576", {})
        achieved = total / (ev * 1e-3) / 1e9
        on_sorted = E.stats().get("sorted_batches", 0) - sorted0 == args.steps
        sustained = None
        if args.leg_sustain_seconds > 0:
            # back-to-back steps for a few seconds: a 20-step region is ~17 ms,
            # so a clock transient moves it; this is the settled rate
            E.sync()
            E.timer_start()
            n_s, t_s = 0, time.perf_counter()
            while time.perf_counter() - t_s < args.leg_sustain_seconds:
                for _ in range(50):
                    E.device_batch(data, d_off, d_len, R, out, total_bytes=total, asynchronous=True)
                n_s += 50
                E.sync()
            s_ms = E.timer_stop() / n_s
            s_gbs = total / (s_ms * 1e-3) / 1e9
            sustained = {"steps": n_s, "step_ms": round(s_ms, 4), "achieved_gb_s": round(s_gbs, 1),
                         "frac": round(s_gbs / HBM_PEAK_GBS, 4),
                         "digest_unchanged": E.crc32c_device(out, R * 4) == dig}
        cpu = None
        if not args.no_cpu:
            # the reference over the first records of the same batch (<= 1 GiB,
            # host DRAM), on every CPU this process may use
            from oracle.oracle import Oracle, Reference, reference_available
            if reference_available():
                usable, cpus = usable_cpus()
                k = int(np.searchsorted(np.cumsum(ln, dtype=np.uint64), np.uint64(1 << 30)))
                nb = int(off[k - 1] + ln[k - 1])
                hb = Oracle().fill(nb, W.DATA_SEED, 0)
                ref = Reference()
                want = ref.batch(hb, off[:k], ln[:k], threads=usable)
                rate, passes = timed_rate(lambda: ref.batch(hb, off[:k], ln[:k], threads=usable),
                                          nb, args.leg_cpu_seconds)
                rate1, _ = timed_rate(lambda: ref.batch(hb, off[:k // 8], ln[:k // 8], threads=1),
                                      int(off[k // 8]), args.leg_cpu_seconds / 2)
                got = out.download(np.uint32, k)
                cpu = {"value": round(rate, 2), "unit": "GiB/s", "cores": usable,
                       "kind": "reference", "single_thread_value": round(rate1, 2),
                       "sample": f"records 0..{k - 1} of the same batch ({nb / 2**30:.3f} GiB, host "
                                 f"DRAM), consus::crc32c from common/crc32c.cc compiled unmodified, "
                                 f"{passes} passes x {usable} std::threads; single thread over "
                                 f"records 0..{k // 8 - 1}; cpu: {cpus['model']}",
                       "matches_gpu": bool(np.array_equal(got, want))}
        res.update({
            "metric": "GiB/s CRC32C over device-resident mixed-length records (Zipf 64 B-64 KiB)",
            "value": round(total / (wall) / 2**30, 2), "unit": "GiB/s",
            "ms_per_step": round(wall * 1e3, 4),
            "data": "synthetic: config-3 Zipf lengths, splitmix64 stream 0xDA7A5EED in HBM",
            "config": {"workload": f"{R} mixed-length records, device-resident, 1 x MI355X "
                                   f"(BASELINE.json configs[2])", "total_bytes": total},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic[0] is None else round(traffic[0]),
                         "traffic_note": traffic[1], "algorithmic_bytes": total,
                         "step_ms_events": round(ev, 4),
                         "kernel": ("sorted_cost_kernel + crc32c_sorted_kernel (whole step, "
                                    "sorted path)") if on_sorted else
                                   "plan + crc32c_chunk_kernel + finalize (whole step, piece path)"},
            "digest_verified": (dig == g.get("digest")) if g and R == 1 << 20 else None,
            "digests": [f"{dig:#010x}"], "sustained": sustained, "cpu_baseline": cpu})
        return res
    if args.config == "single":
        n = 1 << 32
        gs = gold.get("single_record_seed0xc0de", {}).get("crc", {})
        data = E.DeviceBuffer(n + 4097)
        data.fill_splitmix64(SEED)
        if args.child_pmc:
            for _ in range(PMC_CHILD_STEPS):
                E.crc32c_device(data, n)
            return {}
        for _ in range(args.warmup):
            E.crc32c_device(data, n)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            got = E.crc32c_device(data, n)   # synchronous: kernels, 4-byte read-back
        wall = (time.perf_counter() - t0) / args.steps
        odd = E.crc32c_device(data, n + 4097)
        ok = (got == gs.get(str(n)) and odd == gs.get(str(n + 4097))) if gs else None
        res.update({
            "metric": "GiB/s CRC32C of one device-resident 4 GiB record (consus::crc32c semantics)",
            "value": round(n / wall / 2**30, 2), "unit": "GiB/s", "ms_per_step": round(wall * 1e3, 4),
            "data": "synthetic: splitmix64 stream 0xC0DE in HBM (the cfg-2 bytes as one record)",
            "config": {"workload": "1 x 4 GiB record, device-resident, 1 x MI355X; 1,048,575 "
                                   "aligned 4 KiB chunks through crc32c_span_chunk_kernel (the fixed kernel's code), "
                                   "head/tail windows and a two-level combine tree on the GPU"},
            "roofline": {"bound": "hbm", "achieved": round(n / wall / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(n / wall / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic[0] is None else round(traffic[0]),
                         "traffic_note": traffic[1] + " (crc32c_span_chunk_kernel, per call)",
                         "kernel": "crc32c_span_chunk_kernel + single_tree + single_join "
                                   "(whole call, host sync included)"},
            "digest_verified": ok, "crc": f"{got:#010x}"})
        return res
    # stream / pcie4k: host-resident segments through the H2D -> CRC -> D2H pipeline
    nseg = args.segments or (64 if args.config == "pcie4k" else 16)
    filler = E.DeviceBuffer(W.SEGMENT_BYTES + 64)

    def fill(nbytes, byte_off, seed):
        # bytes [byte_off, +nbytes) of a stream, produced on the device (8-byte aligned window)
        a = byte_off & ~7
        n = nbytes + (byte_off - a)
        filler.fill_splitmix64(seed, byte_offset=a, nbytes=(n + 7) & ~7)
        return filler.download(np.uint8, n)[byte_off - a:]
    segs = []
    if args.config == "stream":
        for buf, fo, fl in W.log_segments(nseg, lambda n, o: fill(n, o, W.DATA_SEED)):
            pb = E.PinnedBuffer(buf.size)
            pb.array[:] = buf
            segs.append((pb, fo, fl))
        metric = "GiB/s host-to-host CRC32C of 64 MiB durable-log segments (H2D+CRC+D2H)"
        workload = f"{nseg} x 64 MiB durable-log segments in pinned host memory, 1 x MI355X " \
                   f"(BASELINE.json configs[4])"
    else:
        per = W.SEGMENT_BYTES // RECORD
        for k in range(nseg):
            pb = E.PinnedBuffer(W.SEGMENT_BYTES)
            pb.array[:] = fill(W.SEGMENT_BYTES, k * W.SEGMENT_BYTES, SEED)
            segs.append((pb, np.arange(per, dtype=np.uint64) * RECORD,
                         np.full(per, RECORD, dtype=np.uint32)))
        metric = "GiB/s host-to-host CRC32C of 4 KiB records starting in pinned host memory"
        workload = f"{nseg * per} x 4 KiB records (config-2 bytes) in pinned host memory, " \
                   f"64 MiB segments, 1 x MI355X"
    maxrec = max(int(fo.size) for _, fo, _ in segs)
    pipe = E.Pipeline(W.SEGMENT_BYTES, maxrec, depth=3)
    outs = [np.zeros(int(fo.size), dtype=np.uint32) for _, fo, _ in segs]
    total = sum(int(pb.nbytes) for pb, _, _ in segs)

    def step():
        ts = [pipe.submit(pb, fo, fl, o) for (pb, fo, fl), o in zip(segs, outs)]
        for t in ts:
            pipe.wait(t)
    if args.child_pmc:
        step()
        pipe.close()
        return {}
    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    wall = (time.perf_counter() - t0) / args.steps
    ok = None
    if args.config == "stream":
        g = gold.get("log_segments_64MiB", {}).get("segments", [])
        dev = E.DeviceBuffer(maxrec * 4)
        digs = []
        for o in outs[:len(g)]:
            dev.upload(o)
            digs.append(E.crc32c_device(dev, o.size * 4))
        ok = bool(g) and all(d == x["digest"] for d, x in zip(digs, g))
    else:
        dev = E.DeviceBuffer(W.SEGMENT_BYTES // RECORD * 4)
        digs = []
        for o in outs:
            dev.upload(o)
            digs.append(E.crc32c_device(dev, o.size * 4))
        from consus_amd.shard import combine_digests
        whole = combine_digests(digs, [o.size for o in outs])
        g = gold.get(f"fixed_4096_seed0xc0de_per_1048576", {})
        ok = (whole == g.get("block_digests", [None])[0]) if nseg * (W.SEGMENT_BYTES // RECORD) \
            == 1 << 20 else None
    pipe.close()
    cpu = None
    if not args.no_cpu:
        # the reference on the same host-resident segments (no link to cross):
        # what txman's own cores would do with these buffers
        from oracle.oracle import Reference, reference_available
        if reference_available():
            usable, cpus = usable_cpus()
            ref = Reference()
            if args.config == "stream":
                frames = sum(int(fl.astype(np.uint64).sum()) for _, _, fl in segs)
                run = lambda th: [ref.batch(pb.array, fo, fl, threads=th) for pb, fo, fl in segs]
                ok_cpu = all(np.array_equal(ref.batch(pb.array, fo, fl, threads=usable), o)
                             for (pb, fo, fl), o in zip(segs, outs))
            else:
                frames = total
                per = W.SEGMENT_BYTES // RECORD
                run = lambda th: [ref.fixed(pb.array, RECORD, RECORD, per, threads=th)
                                  for pb, _, _ in segs]
                ok_cpu = all(np.array_equal(ref.fixed(pb.array, RECORD, RECORD, per, threads=usable),
                                            o) for (pb, _, _), o in zip(segs, outs))
            rate, passes = timed_rate(lambda: run(usable), frames, args.leg_cpu_seconds)
            t1 = time.perf_counter()
            run(1)  # one single-thread pass
            rate1 = frames / 2**30 / (time.perf_counter() - t1)
            cpu = {"value": round(rate, 2), "unit": "GiB/s", "cores": usable, "kind": "reference",
                   "single_thread_value": round(rate1, 2),
                   "sample": f"the same {nseg} pinned host segments ({frames / 2**30:.3f} GiB of "
                             f"checksummed bytes per pass), consus::crc32c from common/crc32c.cc "
                             f"compiled unmodified, {passes} passes x {usable} std::threads, each "
                             f"segment's records split by count; cpu: {cpus['model']}",
                   "matches_gpu": ok_cpu}
    res.update({"metric": metric, "value": round(total / wall / 2**30, 2), "unit": "GiB/s",
                "ms_per_step": round(wall * 1e3, 4),
                "data": "synthetic (SURVEY.md 8(d)); segments pre-built in pinned host memory",
                "config": {"workload": workload, "segments": nseg, "pipeline_depth": 3,
                           "bytes_per_step": total},
                "roofline": {"bound": "pcie", "achieved": round(total / wall / 1e9, 1),
                             "peak": 63.0, "unit": "GB/s",
                             "frac": round(total / wall / 1e9 / 63.0, 4),
                             "traffic": None if traffic[0] is None else round(traffic[0]),
                             "traffic_note": "HBM bytes read by the step's CRC kernels (PMC "
                                             f"FETCH_SIZE): {traffic[1]}; the bound is the host "
                                             "link, PCIe Gen5 x16, 63 GB/s spec",
                             "link_bytes_per_step": total},
                "digest_verified": ok, "cpu_baseline": cpu})
    return res


def run_mid(E, sizes_mib=(1, 4, 16, 20, 64, 128, 256), reps: int = 200) -> dict:
    """Mid-size device batches (VERDICT r4 Next 4; a durable-log segment,
    /root/reference/txman/durable_log.cc:287-347): configs[2]'s record stream
    cut to N MiB, one batch per launch on the engine's own path choice (the
    window path up to 26 MiB / 8192 records, the sorted path above), HIP
    events over `reps` back-to-back batches after a warm-up; every size's
    CRCs checked against the oracle (a checker, outside the timed region)."""
    from consus_amd import workload as W
    from oracle.oracle import Oracle
    off_all, ln_all, _ = W.zipf_records(1 << 20)
    cum = np.cumsum(ln_all, dtype=np.uint64)
    top = int(np.searchsorted(cum, np.uint64(max(sizes_mib)) << np.uint64(20))) + 1
    nbytes = int(cum[top - 1])
    data = E.DeviceBuffer(nbytes + 16)
    data.fill_splitmix64(W.DATA_SEED)
    host = data.download(np.uint8, nbytes)
    d_off, d_len, out = E.DeviceBuffer(top * 8), E.DeviceBuffer(top * 4), E.DeviceBuffer(top * 4)
    O = Oracle()
    rows = []
    try:
        for mib in sizes_mib:
            n = int(np.searchsorted(cum, np.uint64(mib) << np.uint64(20))) + 1
            off, ln = off_all[:n], ln_all[:n]
            total = int(ln.sum(dtype=np.uint64))
            d_off.upload(off)
            d_len.upload(ln)
            st0 = E.stats()
            E.device_batch(data, d_off, d_len, n, out, total_bytes=total)
            st1 = E.stats()
            path = ("window" if st1["window_batches"] > st0["window_batches"] else
                    "sorted" if st1["sorted_batches"] > st0["sorted_batches"] else "other")
            ok = bool(np.array_equal(out.download(np.uint32, n), O.batch(host, off, ln)))
            for _ in range(max(reps // 4, 20)):
                E.device_batch(data, d_off, d_len, n, out, total_bytes=total, asynchronous=True)
            E.sync()
            E.timer_start()
            for _ in range(reps):
                E.device_batch(data, d_off, d_len, n, out, total_bytes=total, asynchronous=True)
            ms = E.timer_stop() / reps
            rows.append({"mib": mib, "records": n, "bytes": total, "us_per_batch": round(ms * 1e3, 2),
                         "gb_s": round(total / (ms * 1e-3) / 1e9, 1), "path": path, "crc_ok": ok})
    finally:
        for b in (data, d_off, d_len, out):
            b.free()
    return {"unit": "us per device batch", "reps": reps,
            "workload": "configs[2] records cut to N MiB, device-resident",
            "batches": rows}


def run_single_split(args, E, dist, rank, world):
    """One record of world x 4 GiB, rank r holding bytes [4 GiB r, 4 GiB (r+1))
    of stream 0xC0DE in its HBM (a record split across GPUs).
    Timed: each rank's synchronous crc32c(0, slice), between barriers, max
    over ranks.  After the timed region the (crc, length) pairs -- 8 bytes
    per rank -- are gathered and folded with the combine operator on rank 0
    (timed once, reported as "exchange_ms") and checked against the golden
    CRC of the whole record."""
    import torch
    from consus_amd import shard
    n = 1 << 32
    start, length = shard.record_slices(world * n, world)[rank]
    data = E.DeviceBuffer(length)
    data.fill_splitmix64(SEED, byte_offset=start)
    for _ in range(args.warmup):
        E.crc32c_device(data, length)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        crc = E.crc32c_device(data, length)  # synchronous: kernels + 4-byte read-back
    dist.barrier()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t[0])
    ranks = rank_identity(E, dist, rank, 0 if args.share_device else
                          int(os.environ.get("LOCAL_RANK", "0")), wall / args.steps * 1e3)
    t1 = time.perf_counter()
    whole = shard.gather_fold(crc, length)
    exch = time.perf_counter() - t1
    if rank == 0:
        gs = golden_digests().get("single_record_seed0xc0de", {}).get("crc", {})
        want = gs.get(str(world * n))
        per = wall / args.steps
        print(json.dumps({
            "metric": "GiB/s CRC32C of one device-resident record split across GPUs "
                      "(consus::crc32c semantics)",
            "value": round(world * n / per / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: splitmix64 stream 0xC0DE, each rank's 4 GiB slice generated in "
                    "its HBM",
            "config": {"workload": f"1 x {world * 4} GiB record, 4 GiB slice per GPU, {world} x "
                                   "MI355X; per-slice crc32c on each GPU, (crc, length) pairs "
                                   "folded with crc32c_combine on rank 0",
                       "parallelism": f"byte slices x{world}, 8-byte exchange after the timed "
                                      "region"},
            "roofline": {"bound": "hbm", "achieved": round(n / per / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(n / per / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "per-rank slice: crc32c_span_chunk_kernel + single_tree + "
                                   "single_join (host sync included)"},
            "exchange_ms": round(exch * 1e3, 3),
            "ranks": ranks, "distinct_gpus": len({r["pci_bus_id"] for r in ranks}),
            "digest_verified": (whole == want) if want is not None else None,
            "crc": f"{whole:#010x}", "cpu_baseline": None}), flush=True)
    dist.destroy_process_group()


def run_zipf_sharded(args, E, dist, rank, world):
    """configs[2]'s record stream continued to world x R records (R = 1M per
    rank), split into contiguous record ranges balanced by BYTES
    (shard.balanced_ranges); rank r generates exactly its
    records' bytes in its HBM and runs the device-resident variable path on
    them.  Timed: the steps between barriers, max over ranks.  Verified: the
    ranks' CRC-vector digests, combined with their record counts, against
    the golden digest of the whole stream prefix (combine of 1M-record block
    digests)."""
    import torch
    from consus_amd import shard
    from consus_amd import workload as W
    R = args.records_per_rank
    n = world * R
    lengths = E.zipf_lengths(W.ZIPF_SEED, n)
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    lo, hi = shard.balanced_ranges(lengths, world)[rank]
    cnt = hi - lo
    start = int(offsets[lo]) if cnt else 0
    a = start & ~7                                  # the fill wants 8-byte aligned offsets
    nbytes = (int(offsets[hi - 1]) + int(lengths[hi - 1]) - a) if cnt else 0
    local_total = int(lengths[lo:hi].sum(dtype=np.uint64))
    data = E.DeviceBuffer(nbytes + 16)
    if nbytes:
        data.fill_splitmix64(W.DATA_SEED, byte_offset=a, nbytes=(nbytes + 7) & ~7)
    d_off, d_len, out = (E.DeviceBuffer(max(cnt, 1) * 8), E.DeviceBuffer(max(cnt, 1) * 4),
                         E.DeviceBuffer(max(cnt, 1) * 4))
    if cnt:
        d_off.upload(offsets[lo:hi] - np.uint64(a))
        d_len.upload(lengths[lo:hi])

    def step(asynchronous):
        if cnt:
            E.device_batch(data, d_off, d_len, cnt, out, total_bytes=local_total,
                           asynchronous=asynchronous)
    for _ in range(args.warmup):
        step(False)
    E.sync()
    dist.barrier()
    E.sync()
    sorted0 = E.stats().get("sorted_batches", 0)
    t0 = time.perf_counter()
    E.timer_start()
    for _ in range(args.steps):
        step(True)
    ev = E.timer_stop()
    E.sync()
    dist.barrier()
    wall = time.perf_counter() - t0
    on_sorted = E.stats().get("sorted_batches", 0) - sorted0 == args.steps
    t = torch.tensor([wall, ev], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, ev_max = float(t[0]), float(t[1])
    dig = E.crc32c_device(out, cnt * 4) if cnt else 0
    ranks = rank_identity(E, dist, rank, 0 if args.share_device else
                          int(os.environ.get("LOCAL_RANK", "0")), ev / args.steps)
    got = [None] * world
    dist.all_gather_object(got, (dig, cnt, local_total, ev, on_sorted))
    if rank == 0:
        blocks = golden_digests().get("zipf_seed0x5eed_data0xda7a5eed_blocks", {})
        bd = blocks.get("block_digests", [])
        ok = None
        if R == 1 << 20 and len(bd) >= world:
            want = shard.combine_digests(bd[:world], [1 << 20] * world)
            ok = shard.combine_digests([g[0] for g in got], [g[1] for g in got]) == want
        total = sum(g[2] for g in got)
        per = wall / args.steps
        # per-GPU rate of the slowest rank: its bytes over its own step time
        achieved = min(g[2] / (g[3] / args.steps * 1e-3) / 1e9 for g in got if g[1])
        print(json.dumps({
            "metric": "GiB/s CRC32C over device-resident mixed-length records (Zipf 64 B-64 KiB)",
            "value": round(total / per / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: config-3 Zipf lengths continued to N x 1M records, splitmix64 "
                    "stream 0xDA7A5EED, each rank's bytes generated in its HBM",
            "config": {"workload": f"{n} mixed-length records sharded by bytes over {world} x "
                                   "MI355X (configs[2] per GPU)",
                       "total_bytes": total, "records_per_rank": [g[1] for g in got],
                       "bytes_per_rank": [g[2] for g in got],
                       "parallelism": f"byte-balanced record shards x{world}, no collective in "
                                      "the timed region"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None,
                         "kernel": ("sorted_cost_kernel + crc32c_sorted_kernel" if all(g[4] for g in got)
                                    else "plan + crc32c_chunk_kernel + finalize") +
                                   " (whole step; the slowest rank's bytes over its own step time)"},
            "digest_verified": ok, "digests": [f"{g[0]:#010x}" for g in got],
            "ranks": ranks, "distinct_gpus": len({r["pci_bus_id"] for r in ranks}),
            "cpu_baseline": None}), flush=True)
    dist.destroy_process_group()


# ---- the default line, compacted (VERDICT r5 Next 1) ----------------------------
# The driver keeps about the last 11.5 KB of the run's output: the whole
# default line must fit well inside it, with configs[2]'s leg last.  The full
# record (per-run arrays, long sample strings, host details) goes to a
# detail file that the line names.
LINE_LIMIT = 6000
# legs in the line's order: the driver's record ends with configs[4] and configs[2]
LEG_ORDER = ("mid_batches", "durable_log", "config1_pcie_inclusive", "config4_stream",
             "config2_zipf")


def _pick(d: dict | None, keys) -> dict | None:
    if d is None:
        return None
    return {k: d[k] for k in keys if k in d}


def _compact_cpu(c: dict | None, sample_chars: int = 120) -> dict | None:
    if not c:
        return c
    r = _pick(c, ("value", "unit", "cores", "kind", "single_thread_value", "matches_gpu", "error"))
    if "sample" in c:
        # the sample's first clause (what was hashed); the rest is in the detail file
        s = c["sample"].split(", consus::crc32c")[0].split("; ")[0].split(" (")[0]
        r["sample"] = s if len(s) <= sample_chars else s[:sample_chars - 3] + "..."
    return r


def _compact_secondary(r: dict) -> dict:
    """configs[2], configs[4] and the PCIe-inclusive leg: value, step time,
    roofline, digest check and the same-run reference CPU rate."""
    if "error" in r and "value" not in r:
        return r
    out = _pick(r, ("metric", "value", "unit", "ms_per_step", "steps", "warmup"))
    out["workload"] = (r.get("config") or {}).get("workload")
    out["roofline"] = _pick(r.get("roofline"), ("bound", "achieved", "peak", "frac", "traffic",
                                                "algorithmic_bytes", "step_ms_events"))
    out["digest_verified"] = r.get("digest_verified")
    if r.get("sustained"):
        out["sustained"] = _pick(r["sustained"], ("steps", "step_ms", "frac", "digest_unchanged"))
    out["cpu_baseline"] = _compact_cpu(r.get("cpu_baseline"), 90)
    out["leg_wall_s"] = r.get("leg_wall_s")
    return out


def _compact_mid(r: dict) -> dict:
    if "batches" not in r:
        return r
    return {"reps": r.get("reps"), "workload": "configs[2] records cut to N MiB",
            "cols": ["mib", "us_per_batch", "gb_s", "path", "crc_ok"],
            "batches": [[b["mib"], b["us_per_batch"], b["gb_s"], b["path"], b["crc_ok"]]
                        for b in r["batches"]],
            "leg_wall_s": r.get("leg_wall_s")}


def _compact_dlog(r: dict) -> dict:
    """Per workload and engine: appends/s median, q1, q3 and the medians of the
    runs' p50 / p99 durable latency; the GPU engine against each other engine;
    the median GPU run's per-flush phases."""
    if "workloads" not in r:
        return r
    out = _pick(r, ("value", "unit", "steps", "digest_verified"))
    out["metric"] = "durable-log appends/s, 8 appending threads"
    out["cols"] = "appends/s median, durable-latency us p50 p99 (IQRs: detail file)"
    for wname, w in r["workloads"].items():
        e = {name: [round(s["appends_per_s"]["median"])] +
             [round(s["durable_latency_us"][q]) for q in ("p50_median", "p99_median")]
             for name, s in w["engines"].items()}
        f = w.get("flush", {})
        out[wname] = {
            "engines": e,
            "gpu_vs": {k: [v["appends_ratio"], v["beyond_spread"].replace(" run spread", "")]
                       for k, v in w.get("gpu_vs", {}).items()},
            "flush": dict(_pick(f, ("flushes", "host_flushes", "frame_bytes_per_flush",
                                    "batch_crc_vs_bound")),
                          us_per_flush=_pick(f.get("us_per_flush", {}), ("batch_crc", "pwrite")))}
    out["cpu_baseline"] = "engines.reference-scheme (the detail file has it in full)"
    out["leg_wall_s"] = r.get("leg_wall_s")
    return out


def compact_line(rec: dict, detail: str | None) -> dict:
    """The default line as printed: the headline keys unchanged, the legs
    compacted and in LEG_ORDER (configs[2] last), `detail_file` naming the
    full record."""
    line = {k: v for k, v in rec.items() if k not in LEG_ORDER}
    if line.get("cpu_baseline"):
        c = dict(line["cpu_baseline"])
        c.pop("host", None)  # in the detail file; the sample names the CPU model
        c.pop("first_crc", None)
        line["cpu_baseline"] = c
    if detail:
        line["detail_file"] = detail
    for k in LEG_ORDER:
        if k not in rec:
            continue
        r = rec[k]
        if k == "mid_batches":
            line[k] = _compact_mid(r)
        elif k == "durable_log":
            line[k] = _compact_dlog(r)
        else:
            line[k] = _compact_secondary(r)
    return line


def _clip_strings(x, n: int):
    """Every string inside x cut to n characters (error texts, samples)."""
    if isinstance(x, str):
        return x if len(x) <= n else x[:n - 3] + "..."
    if isinstance(x, dict):
        return {k: _clip_strings(v, n) for k, v in x.items()}
    if isinstance(x, list):
        return [_clip_strings(v, n) for v in x]
    return x


def fit_line(line: dict) -> dict:
    """Keep the printed line under LINE_LIMIT whatever the legs carry (a
    failing leg's error text, say): long strings are clipped first, then the
    durable-log leg keeps only its headline ratios; configs[2] stays last."""
    if len(json.dumps(line)) <= LINE_LIMIT:
        return line
    line = _clip_strings(line, 160)
    if len(json.dumps(line)) > LINE_LIMIT and isinstance(line.get("durable_log"), dict):
        d = line["durable_log"]
        slim = {k: d[k] for k in ("value", "unit", "digest_verified", "error") if k in d}
        slim.update({w: {"gpu_vs": v.get("gpu_vs")} for w, v in d.items()
                     if isinstance(v, dict) and "gpu_vs" in v})
        rest = {k: v for k, v in line.items() if k not in LEG_ORDER}
        rest.update({k: (slim if k == "durable_log" else line[k]) for k in LEG_ORDER if k in line})
        line = rest
    if len(json.dumps(line)) > LINE_LIMIT:
        line = _clip_strings(line, 60)
    return line


def write_detail(rec: dict) -> str | None:
    """The full record (every run, every sample string) to BENCH_DETAIL, by
    default gpurun_out/bench_detail.json; returns the path the line names."""
    path = os.environ.get("BENCH_DETAIL", os.path.join(REPO, "gpurun_out", "bench_detail.json"))
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(rec, f)
            f.write("\n")
    except OSError as e:
        progress(f"detail file not written: {e}")
        return None
    return os.path.relpath(path, REPO) if os.path.abspath(path).startswith(REPO) else path


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not args.child_pmc:
        if world == 1 and args.gpus > 1:
            sys.exit("for --gpus N>1 launch with torch.distributed.run (one process per GPU)")
    if args.records_per_rank is None:
        args.records_per_rank = (2 << 20) if world > 1 and args.config == "fixed4k" else 1 << 20

    # Traffic pass first, before this process touches the GPU.
    traffic, traffic_note = (None, "skipped")
    if rank == 0 and world == 1 and not args.child_pmc and not args.no_pmc and \
            args.config in ("fixed4k", "zipf", "single", "stream", "pcie4k"):
        progress(f"PMC traffic pass ({args.config})")
        traffic, traffic_note = pmc_traffic(args)
    # The other single-GPU BASELINE configs ride in the headline line (N = 1):
    # configs[2], configs[4] and configs[1]'s bytes starting in host memory.
    legs = []
    if world == 1 and args.config == "fixed4k" and not args.child_pmc and not args.no_legs:
        for key, cfg in (("config2_zipf", "zipf"), ("config4_stream", "stream"),
                         ("config1_pcie_inclusive", "pcie4k")):
            # the zipf leg warms up for >= 100 steps (~80 ms): it starts after host-side
            # preparation with the GPU idle, and 5 steps leave it in the clock ramp;
            # it times >= 100 steps (~77 ms, sync-bracketed), since in a 20-step window
            # (15 ms) the restart after the warm-up's sync costs ~6 us a step
            # (round 5, profiles/r05_zipf_leg_window.txt)
            sub = sub_args(args, cfg, **({"warmup": max(args.warmup, 100), "steps": max(args.steps, 100)}
                                         if cfg == "zipf" else {}))
            progress(f"PMC traffic pass ({cfg})")
            legs.append((key, sub, pmc_traffic(sub) if not args.no_pmc else (None, "skipped")))
        # the durable-log front-end: appends/s and the per-flush
        # GPU batch against its bound, beside the reference CPU checksum
        legs.append(("durable_log", sub_args(args, "dlog", steps=30), (None, "n/a")))

    if args.config == "dlog":  # a child process drives the engine; none here
        if rank == 0:
            print(json.dumps(run_dlog(args)), flush=True)
        return

    # The engine is loaded before torch so both bind the /opt/rocm HIP runtime.
    import consus_amd as E
    progress("engine init")
    E.init(0 if args.share_device else local)
    if args.config != "fixed4k" and not (args.config in ("single", "zipf") and world > 1):
        if world != 1:
            sys.exit("secondary configs other than single and zipf run on one GPU")
        res = run_secondary(args, E, (traffic, traffic_note))
        if not args.child_pmc:
            print(json.dumps(res), flush=True)
        return

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # gloo prints its connection census on fd 1; keep stdout for the JSON line
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    if args.config == "single":  # world > 1: one record split across the ranks
        run_single_split(args, E, dist, rank, world)
        return
    if args.config == "zipf":  # world > 1: the record stream sharded by bytes
        run_zipf_sharded(args, E, dist, rank, world)
        return

    R, L = args.records_per_rank, args.record_bytes
    data = E.DeviceBuffer(R * L)
    out = E.DeviceBuffer(R * 4)
    data.fill_splitmix64(SEED, byte_offset=rank * R * L)

    if args.child_pmc:
        for _ in range(3):
            E.device_batch_fixed(data, L, L, R, out)
        return

    for _ in range(args.warmup):
        E.device_batch_fixed(data, L, L, R, out)
    E.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    E.sync()
    t0 = time.perf_counter()
    E.timer_start()
    for _ in range(args.steps):
        E.device_batch_fixed(data, L, L, R, out, asynchronous=True)
    ev_ms = E.timer_stop()          # HIP events on the launch stream (synchronizes it)
    E.sync()
    barrier()
    wall = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([wall, ev_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ev_ms_max = float(t[0]), float(t[1])
    else:
        ev_ms_max = ev_ms

    ranks = rank_identity(E, dist, rank, 0 if args.share_device else local, ev_ms / args.steps)
    # Digest of this rank's CRC vector, computed on the GPU: crc32c(0, LE bytes).
    crcs_dev_digest = E.crc32c_device(out, R * 4)
    digests = [crcs_dev_digest]
    if dist is not None:
        g = [None] * world
        dist.all_gather_object(g, crcs_dev_digest)
        digests = g

    do_gather = dist is not None and not args.no_gather and not args.share_device
    if rank != 0:
        g = rccl_gather(E, dist, rank, world, out, R, digests, None) if do_gather else None
        dist.destroy_process_group()
        if g and g.get("error"):
            sys.exit(4)
        return

    # golden digests of 1M-record blocks; a rank holding k whole blocks is
    # checked against their combine (digest(A||B) = Z_4|B|(digest A) ^ digest B),
    # which covers BASELINE configs[3] (2M records per GPU at N = 8)
    blk = 1 << 20
    gold = golden_digests().get(f"fixed_{L}_seed{SEED:#x}_per_{blk}", {})
    verified = None
    exp = gold.get("block_digests", [])
    if exp and R % blk == 0 and world * (R // blk) <= len(exp):
        from consus_amd.shard import combine_digests
        k = R // blk
        want = [combine_digests(exp[i * k:(i + 1) * k], [blk] * k) for i in range(world)]
        verified = all(digests[i] == want[i] for i in range(world))

    # Sustained rate, outside the timed region: back-to-back launches for a
    # few seconds (the per-launch rate must not droop with clocks or power;
    # it also keeps the GPU busy long enough for a utilisation sampler).
    sustained = None
    progress("timed steps done; sustained leg")
    if args.sustain_seconds > 0:
        E.sync()
        E.timer_start()
        n_s, t_s = 0, time.perf_counter()
        while time.perf_counter() - t_s < args.sustain_seconds:
            for _ in range(100):
                E.device_batch_fixed(data, L, L, R, out, asynchronous=True)
            n_s += 100
            E.sync()
        s_ms = E.timer_stop()
        s_gbs = n_s * R * L / (s_ms * 1e-3) / 1e9
        sustained = {"launches": n_s, "seconds": round(s_ms * 1e-3, 3),
                     "launch_ms": round(s_ms / n_s, 4), "achieved_gb_s": round(s_gbs, 1),
                     "frac": round(s_gbs / HBM_PEAK_GBS, 4)}
        if crcs_dev_digest != E.crc32c_device(out, R * 4):
            sustained["error"] = "CRC vector changed under sustained launches"

    # the other single-GPU configs, while the clocks are warm (their CPU legs
    # run after their own GPU timing)
    leg_res = {}
    for key, sub, tr in legs:
        t_leg = time.perf_counter()
        try:
            progress(f"leg {key}")
            r = run_dlog(sub, compact=True) if sub.config == "dlog" else run_secondary(sub, E, tr)
            for k in ("n_gpus", "higher_is_better", "scaling", "vs_baseline", "dtype"):
                r.pop(k, None)
        except Exception as e:  # noqa: BLE001 -- a leg must not lose the headline line
            r = {"error": f"{type(e).__name__}: {e}"[:300]}
        r["leg_wall_s"] = round(time.perf_counter() - t_leg, 2)
        leg_res[key] = r
    if legs:
        t_leg = time.perf_counter()
        try:
            progress("leg mid_batches")
            r = run_mid(E)
        except Exception as e:  # noqa: BLE001
            r = {"error": f"{type(e).__name__}: {e}"[:300]}
        r["leg_wall_s"] = round(time.perf_counter() - t_leg, 2)
        leg_res["mid_batches"] = r

    total_bytes = world * R * L * args.steps
    value = total_bytes / wall / 2**30
    # per-GPU kernel rate; at N > 1 from the slowest rank's launches
    per_launch_ms = ev_ms_max / args.steps
    achieved = R * L / (per_launch_ms * 1e-3) / 1e9
    rec = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: splitmix64(0xC0DE ^ word) stream, generated in HBM before timing "
                "(SURVEY.md 8(d))",
        "config": {
            "workload": f"{R} x {L} B records per GPU, device-resident, {world} x MI355X "
                        + ("(BASELINE.json configs[1])" if world == 1 else
                           "(BASELINE.json configs[3] at N = 8: 16M x 4 KiB records)"
                           if world * R == 16 << 20 else "(configs[3] shape)"),
            "records_per_rank": R, "record_bytes": L, "global_batch": world * R,
            "parallelism": f"record shards x{world}, no collective in the timed region",
        },
        "pct_hbm_peak": round(100.0 * achieved / HBM_PEAK_GBS, 2),
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None if traffic is None else round(traffic),
            "algorithmic_bytes": R * L, "kernel": KERNEL_NAME,
            "launch_ms": round(per_launch_ms, 4), "traffic_note": traffic_note,
        },
        "digest_verified": verified,
        "digests": [f"{d:#010x}" for d in digests],
        "sustained": sustained,
    }
    if world == 1 and not args.no_cpu:
        progress("CPU baseline")
        rec["cpu_baseline"] = cpu_baseline(args)
    else:
        rec["cpu_baseline"] = None
    rec.update(leg_res)
    code = 0
    if world > 1:
        rec["roofline"]["launch_ms_rank0"] = round(ev_ms / args.steps, 4)
        # the ranks' identities first: a hung gather's watchdog prints this line
        multi_rank_fields(rec, ranks, None, world, args.share_device)
        gather = rccl_gather(E, dist, rank, world, out, R, digests, rec) if do_gather else None
        code = multi_rank_fields(rec, ranks, gather, world, args.share_device)
    if leg_res:
        rec = fit_line(compact_line(rec, write_detail(rec)))
    print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if code:
        sys.exit(code)


if __name__ == "__main__":
    main()
