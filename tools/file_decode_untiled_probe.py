"""Untiled fused file decode (RSAMD_FILE_DECODE=0 forces it) of a 4 GiB file from 4+2 shards with
2 missing data shards ({0,1}), fraction of 8 TB/s (4*S read + file written).  RSAMD_LIB_OVERRIDE
loads another build of librsamd.so for A/B."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "java-reed-solomon-distributed-file-system_amd"))
import torch, rsamd
from rsamd import _lib, device as rdev
from rsamd.device import StripeLayout
from rsamd.layout import decode_file_dev, encode_file_dev, file_layout
if os.environ.get("RSAMD_LIB_OVERRIDE"):
    _lib.LIB_PATH = os.environ["RSAMD_LIB_OVERRIDE"]
st = torch.cuda.current_stream()
rs = rsamd.ReedSolomon.create(4, 2)
n = (4 << 30) // 4000 * 4000
_, S = file_layout(rs, n, 1000)
stride = (S + 255) // 256 * 256
f = torch.empty(n, dtype=torch.uint8, device="cuda:0")
rdev.fill_synthetic(f.data_ptr(), 1, StripeLayout(1, n, n, n), 0x5EED, 0, st)
sh = torch.empty(6 * stride, dtype=torch.uint8, device="cuda:0")
encode_file_dev(rs, f.data_ptr(), n, sh.data_ptr(), stride, 1000, stream=st)
g = torch.empty(n, dtype=torch.uint8, device="cuda:0")
fn = lambda: decode_file_dev(rs, sh.data_ptr(), S, stride, [0, 0, 1, 1, 1, 1], g.data_ptr(), n, 1000, stream=st)
for _ in range(5): fn()
torch.cuda.synchronize()
assert torch.equal(f, g)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record(st)
for _ in range(10): fn()
e.record(st); torch.cuda.synchronize()
t = s.elapsed_time(e) / 10 * 1e-3
print(json.dumps({"file_decode_untiled_01": round((4 * S + n) / t / 8e12, 4)}))
