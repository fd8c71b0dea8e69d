"""The display kernels' branch-free colormap (csrc/display_common.hpp colormap_rgb: one paired-stop
LUT read, roundf + `as u8` as floor(v + 0.5) with the v < 0.5 case) equals the oracle's
display.rs:24-42 restatement on EVERY 32-bit pattern (finite, infinite, NaN, negative): the
identity the render kernels' byte-exactness rests on, proved here rather than sampled."""
import os
import subprocess

import oracle_ffi
from oracle_ffi import _LIB_PATH as LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_colormap_rgb_equals_oracle_on_every_float(tmp_path):
    oracle_ffi.lib()  # built on first use
    exe = tmp_path / "colormap_check"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                           "-I", os.path.join(ROOT, "multi-spectrogram-viewer_amd", "csrc"),
                           os.path.join(ROOT, "tests", "colormap_check.cpp"), "-o", str(exe), "-ldl", "-pthread"])
    out = subprocess.check_output([str(exe), LIB_PATH, "1"], text=True, timeout=600).split()
    n, bad = int(out[0]), int(out[1])
    assert n == 1 << 32
    assert bad == 0
