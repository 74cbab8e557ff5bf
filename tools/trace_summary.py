"""Summarise the headline kernel's dispatches from a rocprofv3 kernel trace
and set them beside bench.py's in-run HIP-event launch time (dev tool).

python tools/trace_summary.py gpurun_out/prof_r01 > profiles/r01_fixed4k_kernel_trace_summary.txt
"""
import csv
import json
import os
import statistics
import sys

d = sys.argv[1]
trace = list(csv.DictReader(open(os.path.join(d, "rocprof_fixed4k", "k_kernel_trace.csv"))))
trace.sort(key=lambda r: int(r["Start_Timestamp"]))


def durations(tag):
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in trace
            if tag in r["Kernel_Name"]]


big = durations("crc32c_fixed_pipe_kernel<4, false>")  # the record batches
small = durations("crc32c_span_chunk_kernel")           # the digest's 4 KiB span
bench = {}
for line in open(os.path.join(d, "rocprof_fixed4k.log")):
    if line.startswith("{"):
        bench = json.loads(line)
print("# rocprofv3 --kernel-trace of: bench.py --config fixed4k --no-cpu --no-pmc --sustain-seconds 0 --steps 30 --warmup 300")
print(f"# crc32c_fixed_pipe_kernel<4, false>: {len(big)} dispatches over the 1M x 4 KiB batch "
      f"(300 warmup + 30 timed);\n# the digest check after timing runs the same code over the 4 MiB "
      f"CRC vector as\n# crc32c_span_chunk_kernel (launch_single): {len(small)} "
      f"dispatch(es).")
print(f"1M x 4 KiB dispatches: n={len(big)} mean={statistics.mean(big):.1f} us "
      f"median={statistics.median(big):.1f} us min={min(big):.1f} us max={max(big):.1f} us")
t = big[-30:]
print(f"timed 30 (the last 30 dispatches): mean={statistics.mean(t):.1f} us  -> bench.py in-run HIP events: "
      f"launch_ms {bench.get('roofline', {}).get('launch_ms')}")
if small:
    print(f"digest dispatches: {statistics.mean(small):.1f} us")
