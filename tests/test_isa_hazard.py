"""Static guard over the built device code (no GPU): no packed f32 VALU instruction directly after a
wide vector-memory store overwrites that store's data registers (the gfx950 / hipcc 7.2 hazard that
corrupted every second float of a dy store in round 2; tools/isa_hazard_check.py)."""
import glob
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not glob.glob(os.path.join(ROOT, "build", "*.o")) or not shutil.which("objcopy")
                    or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built objects (make) and ROCm's llvm tools")
def test_no_packed_valu_overwrites_wide_store_data():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_hazard_check.py"), os.path.join(ROOT, "build")],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    assert "0 hazard(s)" in p.stdout


def test_no_bitcast_of_vector_lane_lvalues():
    """ROCm 7.2's clang reads element 0 for `__builtin_bit_cast(T, v[i])` on an ext_vector_type lvalue (the
    root cause of round 4's wrong pooled-dz dy, tools/bitcast_lane_probe.cpp): no source may contain one."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_hazard_check.py"), "--bitcast-lanes"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout[-4000:]
    assert "0 bit_cast lane finding(s)" in p.stdout
