"""Debug helper: persistent vs launch W64 routes under a rule program."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
import torch
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.router.rules import RuleSet
from ccfd_demo_summit_amd.engine import StreamEngine
from ccfd_demo_summit_amd.ops.kernels import DeviceModel, DeviceRules
from ccfd_demo_summit_amd.contracts import decode_wire, encode_wire

gpu = torch.device("cuda", 0)
X, _ = generate(4096 * 6, seed=12)
m = build_model("mlp", seed=4, X_ref=X[:20000], calibrate_rate=0.05)
for text in ["when amount > 200 and proba >= 0.2 then fraud\notherwise standard",
             "when V17 < -2.5 or abs(V14) > 4 then fraud\notherwise standard",
             "when proba >= 0.2 then fraud\notherwise standard",
             "when amount > 200 then fraud\notherwise standard",
             "when Time > 50000 then fraud\notherwise standard"]:
    rs = RuleSet.parse(text)
    out = {}
    for mode in ("launch", "persistent"):
        eng = StreamEngine(DeviceModel(m, gpu, wire=True), batch=4096, depth=4, streams=2, input_mode="zerocopy",
                           exec_mode=mode, rules=DeviceRules(rs, gpu))
        out[mode] = eng.score(X)
        eng.close()
    Xs = decode_wire(encode_wire(X))
    for mode, (p, r) in out.items():
        want = rs.evaluate(p, X=Xs)
        bad = np.nonzero(r != want)[0]
        print(repr(text.splitlines()[0]), mode, "mismatch", len(bad), "rows", bad[:8].tolist(),
              "r", r[bad[:8]].tolist(), "rowmod16", sorted(set((bad % 16).tolist()))[:16])
    print("  p equal launch/persist:", np.array_equal(out["launch"][0], out["persistent"][0]))
