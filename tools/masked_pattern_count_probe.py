"""10+4 x 4 MiB x 128 per-stripe-pattern decode (device bitmasks), 4 erasures per stripe, with the
stripes' patterns drawn at random from a pool of P distinct patterns: P = 1 is the uniform case,
P = 1001 every 4-erasure pattern.  Few patterns = few table records (scalar-cache hits) but still
mixed shard sets per stripe; the curve separates the two costs.  Fraction of 8 TB/s."""
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
allpats = np.array([[i not in c for i in range(k + m)] for c in itertools.combinations(range(k + m), 4)])
rng = np.random.default_rng(0)
flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
res = {}
for P in [int(x) for x in os.environ.get("PROBE_P", "1,2,4,16,128,1001").split(",")]:
    pool = allpats[rng.choice(len(allpats), P, replace=False)]
    present = pool[rng.integers(0, P, B)]
    bits = torch.from_numpy(rdev.presence_bits(present).view(np.int32)).cuda()
    fn = lambda: rdev.decode_masked_bits(rs, buf.data_ptr(), bits.data_ptr(), lay, 0, st)
    for _ in range(int(os.environ.get("PROBE_WARM", "1"))): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(5): fn()
    e.record(st); torch.cuda.synchronize()
    t = s.elapsed_time(e) / 5 * 1e-3
    if os.environ.get("PROBE_PER_ITER"):  # one event pair per call: is the slow leg slow throughout?
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
        ev[0].record(st)
        for i in range(10):
            fn(); ev[i + 1].record(st)
        torch.cuda.synchronize()
        res[f"P{P}#{len(res)}_per_call"] = [round(14 * S * B / (ev[i].elapsed_time(ev[i + 1]) * 1e-3) / 8e12, 3)
                                            for i in range(10)]
    rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    assert int(flag.item()) == 0
    res[f"P{P}#{len(res)}"] = round(14 * S * B / t / 8e12, 4)
print(json.dumps(res))
