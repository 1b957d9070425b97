"""Pack a real NPKit dump of the product as a CPU fixture for msccl_amd/npkit.py:

    MSCCL_AMD_NPKIT=1 NPKIT_DUMP_DIR=gpurun_out/nk/dump python tools/npkit_capture.py   (GPU box)
    python tests/golden/make_npkit_golden.py gpurun_out/nk/dump

writes tests/golden/npkit/dump.tar.gz (2 ranks, 4 launches of a 2-rank all-pairs LL AllReduce).
The reference's trace generator was not run on it: executing it here was refused (DESIGN.md,
"Parity pins"), so the converter's expected values come from hand-worked cases instead."""
import os
import sys
import tarfile

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "npkit")


def main(dump_dir: str) -> None:
    os.makedirs(HERE, exist_ok=True)
    with tarfile.open(os.path.join(HERE, "dump.tar.gz"), "w:gz") as t:
        for f in sorted(os.listdir(dump_dir)):
            t.add(os.path.join(dump_dir, f), arcname=f)


if __name__ == "__main__":
    main(sys.argv[1])
