"""Kernel-trace probe: resident + lineage GLM passes issued on two streams (inspect the
start/end timestamps in the rocprofv3 kernel trace to see whether they overlap)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["O3S_GLM_OVERLAP"] = "0"
from orange3_spark_amd import Session, SessionConf  # noqa: E402
from orange3_spark_amd.ml import common as U  # noqa: E402
from orange3_spark_amd.models import glm as GLM  # noqa: E402
from orange3_spark_amd.ops import glm as G  # noqa: E402

s = Session(SessionConf().set("o3s.device", "cuda"))
df = s.synthetic.classification(int(float(os.environ.get("ROWS", "2e8"))), 256, seed=7, resident_fraction=0.15)
data = GLM.GlmData(s.comm, U.features_column(df, "features"), U.numeric_column(df, "label", torch.float32), None)
dev = data.device
cf = torch.zeros(data.ws.dpad + 1, dtype=torch.float32, device=dev)
spec, r0, nl = data.lineage
cus = torch.cuda.get_device_properties(dev).multi_processor_count
ws_r = G.GlmWorkspace(dev, data.ld, grid=cus * 2)
ws_l = G.GlmWorkspace(dev, data.ld, grid=cus)
side = torch.cuda.Stream(dev)
for _ in range(3):
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        G.glm_grad_synth(nl, data.ld, spec.d, spec.seed, r0, spec.wtrue, spec.btrue, cf, None, 0, ws_l)
    G.glm_grad(data.X, data.y, None, cf, None, 0, ws_r)
    main.wait_stream(side)
torch.cuda.synchronize()
print("resident", data.X.shape[0], "lineage", nl)
