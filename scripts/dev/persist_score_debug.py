"""Debug helper: StreamEngine.score (synchronous DMA path) under each exec mode / row format."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
import torch
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.engine import StreamEngine
from ccfd_demo_summit_amd.ops.kernels import DeviceModel

gpu = torch.device("cuda", 0)
X, _ = generate(4096 * 6, seed=12)
m = build_model("mlp", seed=4, X_ref=X[:20000], calibrate_rate=0.05)
for wire in (False, True):
    ref = m.wire_proba(X) if wire else m.predict_proba(X, emulate_bf16=True)
    for mode in ("launch", "persistent"):
        for im in ("zerocopy", "dma"):
            eng = StreamEngine(DeviceModel(m, gpu, wire=wire), batch=4096, depth=4, streams=2, input_mode=im,
                               exec_mode=mode)
            p, r = eng.score(X)
            eng.close()
            print(f"wire={wire} {mode} {im}: max|p-ref|={np.abs(p - ref).max():.3g} p.std={p.std():.3g} "
                  f"first={p[:3]}", flush=True)
