"""Time the GLM gradient pass pieces on the bench config: resident rows only, lineage rows
only (each at several grids), and both overlapped on two streams.  One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from orange3_spark_amd import Session, SessionConf  # noqa: E402
from orange3_spark_amd.ml import common as U  # noqa: E402
from orange3_spark_amd.models import glm as GLM  # noqa: E402
from orange3_spark_amd.ops import glm as G  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    n = int(float(os.environ.get("ROWS", "1e9")))
    s = Session(SessionConf().set("o3s.device", "cuda"))
    df = s.synthetic.classification(n, 256, seed=7)
    feat = U.features_column(df, "features")
    y = U.numeric_column(df, "label", torch.float32)
    os.environ["O3S_GLM_OVERLAP"] = "0"
    data = GLM.GlmData(s.comm, feat, y, None)
    dev = data.device
    cf = torch.zeros(data.ws.dpad + 1, dtype=torch.float32, device=dev)
    cf[:256] = 0.01
    spec, r0, nl = data.lineage
    res = {"resident_rows": int(data.X.shape[0]), "lineage_rows": int(nl)}
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    for mult in (1, 2, 3, 8):
        ws = G.GlmWorkspace(dev, data.ld, grid=cus * mult)
        res[f"resident_ms_grid{mult}x"] = timeit(lambda: G.glm_grad(data.X, data.y, None, cf, None, 0, ws))
    for mult in (1, 2, 8):
        ws = G.GlmWorkspace(dev, data.ld, grid=cus * mult)
        res[f"lineage_ms_grid{mult}x"] = timeit(
            lambda: G.glm_grad_synth(nl, data.ld, spec.d, spec.seed, r0, spec.wtrue, spec.btrue, cf, None, 0, ws))
    side = torch.cuda.Stream(dev)
    for rm, lm in ((2, 1), (3, 1), (8, 1), (8, 8), (1, 1), (2, 2)):
        ws_r = G.GlmWorkspace(dev, data.ld, grid=cus * rm)
        ws_l = G.GlmWorkspace(dev, data.ld, grid=cus * lm)

        def both():
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                G.glm_grad_synth(nl, data.ld, spec.d, spec.seed, r0, spec.wtrue, spec.btrue, cf, None, 0, ws_l)
            G.glm_grad(data.X, data.y, None, cf, None, 0, ws_r)
            main.wait_stream(side)
        res[f"overlap_ms_r{rm}x_l{lm}x"] = timeit(both)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
