"""Parameter files (host-only, no GPU): the reference reads ~/.nccl.conf and then /etc/nccl.conf
into the environment before its first parameter read, never overwriting a variable that is
already set (src/misc/param.cc:25-60, called from ncclInit, src/init.cc:70-85).

Each case runs in a child process: setenv there must not leak into this test process."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(code, env_extra=None, tmp_path=None):
    env = dict(os.environ)
    for k in ("NCCL_ALGO", "MSCCL_AMD_REFERENCE_SELECTION", "NCCL_TEST_A", "NCCL_TEST_B", "NCCL_TEST_C"):
        env.pop(k, None)
    env.update(env_extra or {})
    prog = textwrap.dedent("""
        import ctypes, json, sys
        sys.path.insert(0, %r)
        import msccl_amd as M
        libc = ctypes.CDLL(None)
        libc.getenv.restype = ctypes.c_char_p
        def getenv(n):
            v = libc.getenv(n.encode())
            return None if v is None else v.decode()
    """ % ROOT) + textwrap.dedent(code)
    out = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return out.stdout.strip()


def test_set_env_file_parses_like_the_reference(tmp_path):
    conf = tmp_path / "nccl.conf"
    # the first '=' splits; a line without '=' is skipped; an existing variable is kept
    conf.write_text("NCCL_TEST_A=1=2\nno equals sign here\nNCCL_TEST_B=\nNCCL_TEST_C=from-file\n")
    got = _child("""
        r = M.lib().mscclAmdSetEnvFile(%r.encode())
        print(json.dumps([r, getenv("NCCL_TEST_A"), getenv("NCCL_TEST_B"), getenv("NCCL_TEST_C")]))
    """ % str(conf), {"NCCL_TEST_C": "from-env"})
    assert got == '[0, "1=2", "", "from-env"]'


def test_missing_file_is_an_error_only_for_the_explicit_call(tmp_path):
    got = _child("""
        print(M.lib().mscclAmdSetEnvFile(%r.encode()))
    """ % str(tmp_path / "absent.conf"))
    assert got == "2"  # ncclSystemError; initEnv itself skips absent files silently


def test_file_parameters_reach_the_planner(tmp_path):
    """NCCL_ALGO from a parameter file gates MSCCL for AllReduce like the environment does."""
    from msccl_amd import xmlgen
    xml = tmp_path / "ar.xml"
    xml.write_text(xmlgen.allreduce_allpairs(2, 1, "LL"))
    conf = tmp_path / "nccl.conf"
    conf.write_text("NCCL_ALGO=Ring,Tree\n")
    code = """
        before = M.plan_json(%r, 0, 2, M.COLL_ALLREDUCE, 1024, 7, 0, True)["algo"]
        M.lib().mscclAmdSetEnvFile(%r.encode())
        after = M.plan_json(%r, 0, 2, M.COLL_ALLREDUCE, 1024, 7, 0, True)["algo"]
        print(before, after)
    """ % (str(xml), str(conf), str(xml))
    assert _child(code) == "0 -1"
    # the environment wins over the file
    assert _child(code, {"NCCL_ALGO": "MSCCL,Ring"}) == "0 0"
