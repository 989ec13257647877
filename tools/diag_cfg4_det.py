"""cfg-4 determinism probe: two eager and two graph TrainSteps from identical models; prints
per-step losses and the parameters that differ after 2 steps (eager vs eager, eager vs graph)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import importlib  # noqa: E402

pkg = importlib.import_module("music-recommendation-multimodal_amd")
tg = importlib.import_module("test_gpu_text")


def run(graph, steps=2, p=0.1):
    m, bd = tg._cfg4(pkg, seed=3, p=p)
    s = pkg.TrainStep(m, lr=1e-3, use_graph=graph, seed=5)
    losses = [float(s.step(bd)) for _ in range(steps)]
    torch.cuda.synchronize()
    return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}


for p in (0.0, 0.1):
    e1, se1 = run(False, p=p)
    e2, se2 = run(False, p=p)
    g1, sg1 = run(True, p=p)
    print("p", p, "eager", e1, e2, "graph", g1)
    print("  eager-eager differ:", [k for k in se1 if not torch.equal(se1[k], se2[k])][:10])
    print("  eager-graph differ:", [k for k in se1 if not torch.equal(se1[k], sg1[k])][:10])
