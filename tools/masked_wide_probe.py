"""Per-stripe-pattern decode (device bitmasks) of 10+4 x 4 MiB x 128 stripes, 4 erasures per stripe
(random), against the uniform 10+4 decode: fraction of 8 TB/s."""
import itertools, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "java-reed-solomon-distributed-file-system_amd"))
import numpy as np, torch, rsamd
from rsamd import device as rdev
from rsamd.device import StripeLayout
k, m, S, B = 10, 4, 4 << 20, 128
rs = rsamd.ReedSolomon.create(k, m)
lay = StripeLayout.packed(B, k + m, S)
buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
st = torch.cuda.current_stream()
rdev.fill_synthetic(buf.data_ptr(), k, lay, 1, 0, st)
rdev.encode(rs, buf.data_ptr(), lay, st)
rng = np.random.default_rng(0)
present = np.ones((B, k + m), bool)
for t in range(B):
    present[t, rng.choice(k + m, 4, replace=False)] = False
bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).cuda()
def timed(fn, it=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(it): fn()
    e.record(st); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e-3
alg = (k * B + int((~present).sum())) * S
t = timed(lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st))
print(json.dumps({"masked_bits_10_4": round(alg / t / 8e12, 4)}))
# the uniform pattern {0,1,2,3} through the same masked kernel: separates the
# per-stripe record chain from the cost of random patterns
ub = torch.from_numpy(rdev.presence_bits(np.tile(np.arange(14) >= 4, (B, 1))).view(np.int32)).cuda()
t = timed(lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), ub.data_ptr(), lay, 0, st))
print(json.dumps({"masked_bits_uniform_pattern_10_4": round(14 * S * B / t / 8e12, 4)}))
t = timed(lambda: rdev.decode(rs, buf.data_ptr(), [i >= 4 for i in range(14)], lay, st))
print(json.dumps({"uniform_decode_10_4": round(14 * S * B / t / 8e12, 4)}))
