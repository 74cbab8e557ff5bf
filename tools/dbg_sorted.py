import os, sys, itertools, numpy as np
sys.path.insert(0, '/root/repo')
os.environ["MI_CRC32C_VARPATH"] = "sorted"
import consus_amd as E
from oracle.oracle import Oracle
from tests.test_gpu_sorted import _packed, _device_run
E.init(0); orc = Oracle()
def check(lengths, start=0, gap=0, seed=0, inits=None):
    rng = np.random.default_rng(seed)
    lengths = np.array(lengths, dtype=np.uint32)
    offsets, end = _packed(rng, lengths, gap=gap, start=start)
    buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
    got = _device_run(E, buf, offsets, lengths, inits)
    exp = orc.batch(buf, offsets, lengths, inits)
    return [int(i) for i in np.nonzero(got != exp)[0]]
os.environ["MI_CRC32C_SORTED_GRID"] = "1"
for case in ([65536, 4], [65536, 5], [65536, 100], [65536, 200], [65536, 65536], [65536, 4000], [60000, 4], [30000, 4], [8192, 4], [8192, 8192, 4], [1024, 4], [512, 4], [4096, 4, 4, 4],
             [65537], [65536+200], [65536+4000], [65536 + 30000], [65536 + 60000], [65536*2+60000]):
    print(case, check(case), check(case, start=3), check(case, start=64))
