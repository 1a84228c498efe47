"""isParityCorrect over HBM-resident batches (rs_verify_batch_dev): 4+2 x 1 MiB x 4096 and
10+4 x 4 MiB x 128, fraction of 8 TB/s ((k+m)*S*B bytes read).  RSAMD_LIB_OVERRIDE=<path>
loads another build of librsamd.so (A/B of two builds on one box)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "java-reed-solomon-distributed-file-system_amd"))
import torch, rsamd
from rsamd import _lib, device as rdev
from rsamd.device import StripeLayout
if os.environ.get("RSAMD_LIB_OVERRIDE"):
    _lib.LIB_PATH = os.environ["RSAMD_LIB_OVERRIDE"]
st = torch.cuda.current_stream()
flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
res = {}
for k, m, S, B in [(4, 2, 1 << 20, 4096), (10, 4, 4 << 20, 128)]:
    rs = rsamd.ReedSolomon.create(k, m)
    lay = StripeLayout.packed(B, k + m, S)
    buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
    rdev.fill_synthetic(buf.data_ptr(), k, lay, 7, 0, st)
    rdev.encode(rs, buf.data_ptr(), lay, st)
    fn = lambda: rdev.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
    fn(); torch.cuda.synchronize()
    assert int(flag.item()) == 0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(st)
    for _ in range(10): fn()
    e.record(st); torch.cuda.synchronize()
    t = s.elapsed_time(e) / 10 * 1e-3
    res[f"verify_{k}_{m}"] = round((k + m) * S * B / t / 8e12, 4)
    del buf, rs
    torch.cuda.empty_cache()
print(json.dumps(res))
