import sys, time, json, torch
sys.path.insert(0, '/root/repo') if False else None
import os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import __graft_entry__ as ge
ge.build()
from inr_for_audio_amd import _lib
from inr_for_audio_amd.engine import SirenEngine, KanEngine
from inr_for_audio_amd.models import SirenWithSnakeTanh
from inr_for_audio_amd.kan import KAN
lib = _lib.load()
dev = torch.device("cuda:0")
def timeit(eng, steps, prof):
    for _ in range(3): eng.step()
    torch.cuda.synchronize()
    if prof: lib.siren_profile_enable(64 * 100 * 20)
    t0 = time.perf_counter()
    for _ in range(steps): eng.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if prof: lib.siren_profile_enable(0)
    return el / steps * 1e3
res = {}
for name, (H, L, in_dim, n) in {"cfg4": (512, 4, 2, 220160), "cfg2": (1024, 4, 1, 1 << 20)}.items():
    coords = torch.rand(n, in_dim, device=dev) * 2 - 1
    y = torch.sin(2300 * coords[:, 0])
    torch.manual_seed(0)
    m = SirenWithSnakeTanh(in_dim, 1, H, L, 0, 0, first_omega_0=3000.0, hidden_omega_0=30.0)
    eng = SirenEngine(m, coords, y, device=dev, hist_cap=100)
    res[name] = {"noprof": [], "prof": []}
    for r in range(3):
        res[name]["noprof"].append(timeit(eng, 10, False))
        res[name]["prof"].append(timeit(eng, 10, True))
    eng.capture_graph()
    res[name]["graph"] = [timeit(eng, 10, False) for _ in range(3)]
coords = torch.linspace(-1, 1, 441000, device=dev).reshape(-1, 1)
y = torch.sin(2300 * coords[:, 0])
torch.manual_seed(0)
eng = KanEngine(KAN([1, 64, 64, 1]), coords, y, device=dev, hist_cap=100)
res["cfg5"] = {"noprof": [], "prof": []}
for r in range(3):
    res["cfg5"]["noprof"].append(timeit(eng, 10, False))
    res["cfg5"]["prof"].append(timeit(eng, 10, True))
try:
    eng.capture_graph()
    res["cfg5"]["graph"] = [timeit(eng, 10, False) for _ in range(3)]
except Exception as e:
    res["cfg5"]["graph"] = str(e)
print(json.dumps(res))
