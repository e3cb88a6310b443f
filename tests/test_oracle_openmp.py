"""The OpenMP build of the oracle (liboracle_omp.so, bench.py's multi-core CPU figure) returns the
same bits as the serial restatement: rows of the sweeps and of the elementwise steps are
independent, every cell keeps the reference's tap order, and the RNG stays serial."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OMP = os.path.join(ROOT, "oracle", "liboracle_omp.so")

SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import oracle as O
o = O.Filter(plane=O.PLANE_SYNTHETIC, Ny=96, Nz=150, N_min=2, N_max=24, seed=17)
for dt in (1e-8, 1e-8, 1e-5):
    o.filter(dt)
out = {k: o.field(k).tolist() for k in ("u", "v", "w", "T", "rho")}
out["state"] = list(o.rng.state)
print(json.dumps(out))
"""


def _run(lib, threads):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    if lib:
        env["ORACLE_LIB"] = lib
    else:
        env.pop("ORACLE_LIB", None)
    out = subprocess.run([sys.executable, "-c", SCRIPT, os.path.join(ROOT, "oracle")], env=env,
                         capture_output=True, text=True, check=True, timeout=300)
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(not os.path.exists(OMP), reason="liboracle_omp.so not built (make -C oracle)")
def test_openmp_oracle_bit_identical_to_serial():
    ref = _run(None, 1)
    par = _run(OMP, 4)
    assert par["state"] == ref["state"]
    for k in ("u", "v", "w", "T", "rho"):
        assert np.array_equal(np.array(par[k]), np.array(ref[k])), k
