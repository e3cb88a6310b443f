"""The reference's file writers against its own output on its native grid
(tests/golden/writers_native_s42*, made by oracle/gen_golden.py from df.cpp compiled here):

  * filter()'s per-call CSV (df.cpp:466-467, write_csv 764-803): the C-ABI `csv_path` writer
    (df_capi.cpp write_csv_if) on the GPU, and the oracle's writer on the CPU;
  * write_tecplot (df.cpp:712-762) and plot_RST_lerp (677-706) of the C++ drop-in (include/df.hpp)
    through examples/cpp-test.

Headers, line counts and coordinate text are byte-exact (sha256 of the whole coordinate text);
field values agree to 1e-9 relative in the 15-decimal CSV and to the 6 significant digits the
Tecplot writer prints (default ostream precision).
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

FIX = json.load(open(os.path.join(GOLDEN, "writers_native_s42.json")))
NV = 511 * 401  # Tecplot vertex values per coordinate block


def sha(lines):
    return hashlib.sha256("\n".join(lines).encode()).hexdigest()


def check_csv(lines, exact_fields):
    m = FIX["csv"]
    assert lines[0] == m["header"]
    assert len(lines) == m["n_lines"]
    assert sha([",".join(l.split(",")[:2]) for l in lines[1:]]) == m["coord_sha256"]
    for i, ref in m["sample"].items():
        mine = lines[int(i)]
        if exact_fields:
            assert mine == ref, (i, mine, ref)
            continue
        a = [float(x) for x in mine.split(",")]
        b = [float(x) for x in ref.split(",")]
        assert mine.split(",")[:2] == ref.split(",")[:2]
        assert np.allclose(a[2:], b[2:], rtol=1e-9, atol=1e-12), (i, mine, ref)


def test_oracle_csv_writer_native_grid(tmp_path):
    import oracle as O
    o = O.Filter(seed=FIX["seed"])
    for _ in range(FIX["nsteps"]):
        o.filter(FIX["dt"])
    p = tmp_path / "o.csv"
    assert o.write_csv(str(p)) == 0
    check_csv(open(p).read().splitlines(), exact_fields=True)


@pytest.mark.gpu
def test_capi_csv_path_writer_native_grid(tmp_path):
    import dfamd
    p = tmp_path / "cpp_vel_fluc.csv"
    f = dfamd.DigitalFilter(seed=FIX["seed"], device=0, csv_path=str(p))
    for _ in range(FIX["nsteps"]):
        f.filter(FIX["dt"])  # writes the CSV after every call, like df.cpp:466-467
    f.close()
    check_csv(open(p).read().splitlines(), exact_fields=False)


@pytest.mark.gpu
def test_cpp_write_tecplot_and_plot_RST_lerp(tmp_path):
    exe = os.path.join(ROOT, "examples", "cpp-test")
    assert os.path.exists(exe), "examples/cpp-test not built (__graft_entry__.build())"
    run = tmp_path / "run"
    run.mkdir()
    (tmp_path / "files").mkdir()
    tec = tmp_path / "tecplot.dat"
    out = subprocess.run([exe, "writers", str(FIX["seed"]), repr(FIX["dt"]), str(FIX["nsteps"]), str(tec)],
                         cwd=run, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = open(tec).read().splitlines()
    m = FIX["tecplot"]
    assert lines[:3] == m["header"]
    assert len(lines) == m["n_lines"]
    assert sha(lines[3:3 + 2 * NV]) == m["coord_sha256"]
    for i, ref in m["sample"].items():
        i = int(i)
        if i < 3 + 2 * NV:
            assert lines[i] == ref
        else:  # 6 significant digits: equal text, or one unit in the 6th digit at a rounding tie
            a, b = float(lines[i]), float(ref)
            assert lines[i] == ref or abs(a - b) <= 1.5e-5 * abs(b), (i, lines[i], ref)
    for name in ("myRST.csv", "duanRST.csv"):
        mine = open(tmp_path / "files" / name).read()
        assert mine == open(os.path.join(GOLDEN, f"writers_native_s42_{name}")).read(), name
