import sys, os, json, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import bench_configs as B
from distributed_point_functions_amd import kernels, _lib
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
if "c3" in sys.argv: print(json.dumps(B.c3(dev, 2))[:200], flush=True)
n, rec = 1 << 26, 256
gen = torch.Generator(device=dev); gen.manual_seed(4)
db = torch.randint(0, 256, (n * rec,), dtype=torch.uint8, device=dev, generator=gen)
def ck(): return int(db.view(torch.int64).sum().item())
c0 = ck()
for q in (8, 64):
    sel = torch.randint(-2**63, 2**63 - 1, (q * (n // 128), 2), dtype=torch.int64, device=dev, generator=gen)
    ws = torch.empty(max(16, _lib.lib().dpf_amd_inner_product_workspace_size(n, rec, q)), dtype=torch.uint8, device=dev)
    out = torch.empty(q * rec, dtype=torch.uint8, device=dev)
    res = []
    for i in range(4):
        kernels.inner_product(db, n, rec, sel, q, ws, out); torch.cuda.synchronize(); res.append(out.clone())
    print("q", q, "repeat-equal", [bool(torch.equal(res[0], r)) for r in res[1:]], "db unchanged", ck() == c0, flush=True)
