"""Time asp_table_interp3 variants (modes, column counts) on 1e8 points; diagnostic only."""
import sys, time
sys.path.insert(0, "astro-sph-tools_amd")
import numpy as np
import torch
from asp_amd.ionisation import IonisationTable

n = 10 ** 8
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
shape = (41, 141, 49)
axes = [np.linspace(-8.0, 0.0, shape[0]), np.linspace(2.0, 9.0, shape[1]),
        np.concatenate([np.linspace(0.0, 1.0, 21), np.linspace(1.1, 9.0, 28)])]
tab = IonisationTable(rng.uniform(-12.0, 0.0, shape), *axes, redshift_input_index=2)
g = torch.Generator(device=dev); g.manual_seed(0)
st = torch.rand((n, 2), generator=g, device=dev, dtype=torch.float64)
st[:, 0] = st[:, 0] * 8.0 - 8.0
st[:, 1] = st[:, 1] * 7.0 + 2.0
st3 = torch.cat([st, torch.full((n, 1), 2.25, device=dev, dtype=torch.float64)], 1).contiguous()
srt = st[torch.argsort(st[:, 0] * 100 + st[:, 1])].contiguous()
m = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
X = torch.rand(n, generator=g, device=dev, dtype=torch.float64)


def t(name, f, nbytes):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - s) / 5 * 1e3
    print(f"{name:40s} {ms:7.3f} ms  {nbytes / ms / 1e6:7.0f} GB/s", flush=True)


t("copy 40 B/pt (torch)", lambda: torch.add(m, X), n * 24)
t("mode 0, 2 cols", lambda: tab._run(st, 2, 2.25, 0), n * 24)
t("mode 1, 2 cols", lambda: tab._run(st, 2, 2.25, 1, m, X), n * 40)
t("mode 2, 2 cols", lambda: tab._run(st, 2, 2.25, 2, m, X), n * 40)
t("mode 0, 3 cols", lambda: tab._run(st3, 3, 0.0, 0), n * 32)
t("mode 0, 2 cols, sorted states", lambda: tab._run(srt, 2, 2.25, 0), n * 24)
