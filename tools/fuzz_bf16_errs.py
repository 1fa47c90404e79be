import sys, os, tempfile
sys.path.insert(0, '.')
import numpy as np
import die_amd
from die_amd import native
from die_amd.models import fuzz
d = tempfile.mkdtemp()
for seed in range(30):
    blob, shp, used = fuzz.build_random(seed)
    p = os.path.join(d, 'f%d.onnx' % seed); open(p, 'wb').write(blob)
    eng = native.Engine(p, device='hip', max_batch=4, precision='bf16', autotune=False)
    x = np.random.default_rng(seed * 7 + 1).standard_normal((1,) + shp).astype(np.float32)
    ref = native.cpu_run(p, x).reshape(1, -1)
    got = eng.run(x.reshape(1, -1))
    err = float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))
    eng.close()
    print(seed, used, round(err, 4), flush=True)
