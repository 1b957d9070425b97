"""The C-ABI library loads and exports every function include/*.h declares (no GPU calls)."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

import msccl_amd as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?\w+\*?\s+\*?(\w+)\s*\(", text, flags=re.M):
            if m.group(1) not in ("if", "return", "sizeof"):
                names.add(m.group(1))
    return names


def test_all_declared_symbols_exported():
    names = declared_functions()
    assert {"ncclAllReduce", "ncclReduceScatter", "ncclAllGather", "ncclCommInitRank", "ncclCommInitAll",
            "ncclGroupStart", "ncclGroupEnd", "mscclAmdAlgoJson"} <= names
    lib = M.lib()
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.check_output(["nm", "-D", "--defined-only", M.LIB_PATH]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    assert names <= exported


def test_version_and_error_strings():
    assert M.version() == 21212
    lib = M.lib()
    assert lib.ncclGetErrorString(0) == b"no error"
    assert lib.ncclGetErrorString(5) == b"invalid usage"


def test_invalid_arguments_without_gpu():
    lib = M.lib()
    # null comm pointer / invalid comm handle are argument errors, no device call happens
    assert lib.ncclCommInitRank(None, 2, M.UniqueId(), 0) == 4
    assert lib.ncclAllReduce(None, None, 0, 7, 0, None, None) == 4
    assert lib.ncclCommDestroy(None) == 0
    assert lib.ncclGroupEnd() == 5  # not in a group


def test_enum_values_match_reference():
    hdr = open(os.path.join(ROOT, "include", "nccl.h")).read()
    for name, val in [("ncclSum", 0), ("ncclProd", 1), ("ncclMax", 2), ("ncclMin", 3), ("ncclAvg", 4),
                      ("ncclInt8", 0), ("ncclUint8", 1), ("ncclInt32", 2), ("ncclUint32", 3), ("ncclInt64", 4),
                      ("ncclUint64", 5), ("ncclFloat16", 6), ("ncclFloat32", 7), ("ncclFloat64", 8),
                      ("ncclBfloat16", 9), ("ncclInvalidUsage", 5), ("ncclUnhandledCudaError", 1)]:
        assert re.search(r"\b%s\s*=\s*%d\b" % (name, val), hdr), name


def build_c_example(tmp_path):
    """Compile examples/c_allreduce.c against include/nccl.h + libmsccl_amd.so (a C caller written
    for the reference header, as nccl-tests is)."""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "c_allreduce")
    cmd = ["gcc", "-O2", "-Wall", "-Werror", "-I" + os.path.join(root, "include"), "-I/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", os.path.join(root, "examples", "c_allreduce.c"), "-o", exe,
           "-L" + os.path.join(root, "msccl_amd"), "-lmsccl_amd", "-L/opt/rocm/lib", "-lamdhip64",
           "-Wl,-rpath," + os.path.join(root, "msccl_amd"), "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c_caller_compiles_and_links(tmp_path):
    import subprocess
    exe = build_c_example(tmp_path)
    out = subprocess.run([exe, "2", "16", "--version-only"], check=True, capture_output=True, text=True).stdout
    assert "21212" in out
