"""Data-parallel HIP engine on the GPU with the RCCL communicator: weights arrive through
ncclBroadcast, logits leave through ncclAllGather.  A 1-GPU box can only form a world of one rank
(RCCL refuses two ranks on one device), which still runs the whole RCCL path: unique-id exchange
through the DpGroup segment, ncclCommInitRank, broadcast into the parameter arena, all-gather of
logits and decode status, leader D2H of the gathered rows.  Multi-rank DP is covered on the CPU
(tests/test_dp.py) with the same sharding code."""
import json
import os
import urllib.request

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def test_dp_engine_rccl_world1_matches_plain_engine(native, models):
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    plain = native.Engine(path, device="hip", max_batch=8, autotune=False)
    dp = native.Engine(path, device="hip", max_batch=8, autotune=False, dp_world=1,
                       dp_group="die_gpu_dp_%d" % os.getpid())
    info = dp.refresh_info()
    assert info["name"].startswith("dp1(rccl):hip:gfx950")
    for B in (1, 3, 8):
        x = r.synthetic_input(B, cfg, seed=B).reshape(B, -1)
        np.testing.assert_array_equal(dp.run(x), plain.run(x))
    dp.close()
    plain.close()


def test_dp_worker_rccl_world1_http(native, models):
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    wk = native.Worker(path, node_id="dp", max_batch=8,
                       engine={"device": "hip", "dp_world": 1, "dp_group": "die_gpu_dpw_%d" % os.getpid(),
                               "autotune": False})
    ref_eng = native.Engine(path, device="hip", max_batch=8, autotune=False)
    try:
        h = wk.health()
        assert h["engine"]["dp_backend"] == "rccl" and h["engine"]["dp_device_gather"] is True
        res = native.loadgen(port=wk.port, connections=8, requests=64, payload="full", input_numel=3 * 64 * 64)
        assert res["ok"] == 64 and res["failed"] == 0
        x = r.synthetic_input(2, cfg).reshape(2, -1)
        for i in range(2):  # device-decoded text through the DP path == plain engine on parsed floats
            body = json.dumps({"request_id": "g%d" % i, "input_data": [float(v) for v in x[i]]}).encode()
            out = json.loads(urllib.request.urlopen(urllib.request.Request(wk.url + "/infer", data=body),
                                                    timeout=60).read())
            np.testing.assert_array_equal(np.array(out["output_data"], np.float32), ref_eng.run(x[i:i + 1])[0])
        assert wk.health()["device_decoded"] >= 2
    finally:
        wk.stop()
        ref_eng.close()
