"""The RankWork layout guard, on the host (no GPU): every per-type kernel object records the
RankWork layout it was compiled with (devcomm.h: kWorkLayout), and the library refuses to run when
one disagrees with the host code (dispatch.cc: kernelLayoutMismatch, checked at communicator setup
and, right after a variant link, by tools/check_layout.py).  A split layout reads launch arguments
at the wrong offsets: the r05k illegal memory access of a measurement variant (DESIGN.md §10,
tools/lat/README.md) came from a kernel object built with other -D flags than the host objects."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "msccl_amd", "libmsccl_amd.so")

STUB = r"""
#include "device/devcomm.h"
namespace msccl {
#define STUB(N, STAMP) LaunchFn N[6][3] = {}; LaunchFn N##_small[2][4] = {}; LaunchFn N##_fold[4] = {}; \
  LaunchFn N##_pair[4] = {}; LaunchFn N##_two[4] = {}; LaunchFn N##_direct[4] = {};                \
  OneRankFn N##_one = nullptr;                                                                     \
  extern const uint32_t N##_layout = STAMP;
STUB(gLaunch_i8, kWorkLayout) STUB(gLaunch_u8, kWorkLayout) STUB(gLaunch_i32, kWorkLayout)
STUB(gLaunch_u32, kWorkLayout) STUB(gLaunch_i64, kWorkLayout) STUB(gLaunch_u64, kWorkLayout)
STUB(gLaunch_f16, kWorkLayout) STUB(gLaunch_f32, kWorkLayout ^ BAD_F32) STUB(gLaunch_f64, kWorkLayout)
STUB(gLaunch_bf16, kWorkLayout ^ BAD_BF16)
}
extern "C" const char* layoutCheck() { return msccl::kernelLayoutMismatch(); }
"""


def _build(tmp_path, bad_f32, bad_bf16):
    src = tmp_path / "stub.cc"
    src.write_text(STUB)
    out = tmp_path / ("stub_%d_%d.so" % (bad_f32, bad_bf16))
    # -Bsymbolic: the stub's own stamps, not those of a libmsccl_amd.so the process loaded globally
    cmd = ["g++", "-std=c++17", "-shared", "-fPIC", "-O1", "-Wl,-Bsymbolic", "-I", os.path.join(ROOT, "msccl_amd", "csrc"),
           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
           "-DBAD_F32=%d" % bad_f32, "-DBAD_BF16=%d" % bad_bf16, str(src),
           os.path.join(ROOT, "msccl_amd", "csrc", "device", "dispatch.cc"), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("host compiler unavailable: %s" % r.stderr[-300:])
    import ctypes
    lib = ctypes.CDLL(str(out))
    lib.layoutCheck.restype = ctypes.c_char_p
    m = lib.layoutCheck()
    return m.decode() if m else None


def test_layout_check_names_the_stale_object(tmp_path):
    assert _build(tmp_path, 0, 0) is None
    assert _build(tmp_path, 1, 0) == "float32"
    assert _build(tmp_path, 0, 4) == "bfloat16"
    assert _build(tmp_path, 2, 4) == "float32"   # the first stale type in dtype order


def test_built_library_has_one_layout():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_layout
    assert check_layout.mismatch(LIB) is None


def test_variant_scripts_run_the_guard():
    """tools/varbuild.sh and tools/varbuild_full.sh bring the host objects up to date and check the
    linked variant before printing "built"."""
    for name in ("varbuild.sh", "varbuild_full.sh"):
        text = open(os.path.join(ROOT, "tools", name)).read()
        assert "make -s -C msccl_amd/csrc" in text, name
        i = text.index("python3 tools/check_layout.py $OUT")
        assert i < text.index("echo built $OUT"), name
