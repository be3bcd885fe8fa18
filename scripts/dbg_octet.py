import sys; sys.path.insert(0, '/root/repo')
import torch, pyarrow as pa
from igloo_amd.columnar import Column
from igloo_amd.ops._lib import native, ptr, stream
c = Column.from_arrow(pa.array(["abc", "hello", None, "xy"], pa.large_string()), device="cuda:0", dict_encode=False)
pat = torch.tensor([97], dtype=torch.uint8, device="cuda:0")
for fn in (20, 21, 22, 23):
    out = torch.full((4,), 7, dtype=torch.int32, device="cuda:0")
    native().str_fn_int(fn, ptr(pat), 1, ptr(c.offsets), ptr(c.data), 4, ptr(out), stream(out))
    torch.cuda.synchronize()
    print(fn, out.cpu().tolist())
