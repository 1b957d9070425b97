"""Host-only guard for a built library (no GPU): every per-type kernel object must have been compiled
with the RankWork layout of the library's host code (devcomm.h: kWorkLayout, dispatch.cc:
kernelLayoutMismatch).  A kernel object with another layout reads its launch arguments at other
offsets than the host writes them: an illegal memory access on the GPU, not an error code.
Communicator setup refuses such a library; this runs the same check right after a link, so a
measurement variant (tools/varbuild.sh, tools/varbuild_full.sh) fails before it reaches a GPU box.

    python3 tools/check_layout.py path/to/libmsccl_amd.so    # exit 0, or 1 naming the stale type
"""
import ctypes
import sys


def mismatch(path: str):
    lib = ctypes.CDLL(path)
    fn = lib.mscclAmdKernelLayoutMismatch
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    m = fn()
    return m.decode() if m else None


if __name__ == "__main__":
    if len(sys.argv) != 2:
        sys.exit("usage: check_layout.py <library.so>")
    m = mismatch(sys.argv[1])
    if m:
        print("check_layout: %s: the %s kernels were built with another RankWork layout than the host code"
              % (sys.argv[1], m), file=sys.stderr)
        sys.exit(1)
    print("check_layout: %s: every kernel object matches the host's RankWork layout" % sys.argv[1])
