"""Build-time resource check of the gfx950 kernels (no GPU needed).

The Makefile keeps hipcc's `-Rpass-analysis=kernel-resource-usage` report next to every kernel
object (build/obj/device/*.res).  The LL and Simple interpreter kernels of the floating-point
types the benchmarks and the reference's configs use must run without scratch: a spill inside the
FIFO loops is a private-memory round trip per pack, and it cost 10-20 % of LL bandwidth when the
fp16 kernel once needed 1.6 KiB of scratch per lane.  VGPRs must stay <= 128 so that two
512-thread workgroups fit each CU (the schedules' workgroups spin on each other and must all be
resident: __launch_bounds__(512, 4)).
"""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RES = os.path.join(ROOT, "build", "obj", "device")

# mangled element types: f = float, DF16_ = _Float16, NS_4Bf16E = bf16; protocol 0 = LL, 2 = Simple
HOT = re.compile(r"mscclKernelI(f|DF16_|NS_4Bf16E)Li[0-3]ELi[02]EE")


def _kernels():
    out = {}
    for f in glob.glob(os.path.join(RES, "*.res")):
        name = None
        for line in open(f):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
                out[name] = {}
                continue
            m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]): (\d+)", line)
            if m and name:
                out[name]["vgpr" if m.group(1) == "VGPRs" else "scratch"] = int(m.group(2))
    return out


def test_hot_kernels_have_no_scratch_and_fit_two_workgroups_per_cu():
    ks = _kernels()
    if not ks:
        pytest.skip("no kernel resource reports (run __graft_entry__.build() first)")
    hot = {k: v for k, v in ks.items() if HOT.search(k)}
    assert len(hot) == 3 * 4 * 2, sorted(hot)
    for k, v in hot.items():
        assert v.get("scratch", 1) == 0, (k, v)
    for k, v in ks.items():
        # the flat tree's fold kernel runs one or a few workgroups per rank, never co-resident
        # with each other on a CU by necessity, and the two-phase fold one workgroup per CU:
        # __launch_bounds__(512, 1) allows 256 VGPRs
        limit = 256 if "mscclFoldKernel" in k or "mscclTwoPhaseKernel" in k else 128
        # the direct kernel's workgroups never wait on each other (no co-residency needed): its
        # 8-bit forms (4 packs per lane of byte-wise folds) may take up to __launch_bounds__(512, 2)'s
        # 256; the wider types stay at two workgroups per CU
        if re.search(r"mscclDirectKernelI[ah]", k):
            limit = 256
        assert v.get("vgpr", 999) <= limit, (k, v)
        if "mscclDirectKernel" in k:
            assert v.get("scratch", 1) == 0, (k, v)
    fold = {k: v for k, v in ks.items() if re.search(r"mscclFoldKernelI(f|DF16_|NS_4Bf16E)Li[0-3]E", k)}
    assert len(fold) == 3 * 4 * 2, sorted(fold)
    for k, v in fold.items():
        assert v.get("scratch", 1) == 0, (k, v)
    # the small-call kernel (fused exchange inside) for the same types and ops, both argument blocks
    # both transfer sets (devcomm.h: kSetAll, kSetExchange)
    small = {k: v for k, v in ks.items()
             if re.search(r"mscclSmallKernelI(f|DF16_|NS_4Bf16E)Li[0-3]ELi0ELi(2|16)ELi[01]EE", k)}
    assert len(small) == 3 * 4 * 2 * 2, sorted(small)
    for k, v in small.items():
        assert v.get("scratch", 1) == 0, (k, v)
    # the pair kernel (interpreter.h: PairRunner), both argument blocks
    pair = {k: v for k, v in ks.items() if re.search(r"mscclPairKernelI(f|DF16_|NS_4Bf16E)Li[0-3]ELi(2|16)EE", k)}
    assert len(pair) == 3 * 4 * 2, sorted(pair)
    for k, v in pair.items():
        assert v.get("scratch", 1) == 0, (k, v)
    # the two-phase fold (interpreter.h: runTwoPhase), both argument blocks
    two = {k: v for k, v in ks.items() if re.search(r"mscclTwoPhaseKernelI(f|DF16_|NS_4Bf16E)Li[0-3]ELi(2|16)EE", k)}
    assert len(two) == 3 * 4 * 2, sorted(two)
    for k, v in two.items():
        assert v.get("scratch", 1) == 0, (k, v)


# ---------------------------------------------------------------------------------------------
# Inline asm that issues a vector- or scalar-memory instruction takes VGPR inputs only.  The
# compiler's hazard recognizer does not insert the "VALU writes an SGPR, VMEM reads it" wait states
# for operands of inline asm: a wave-uniform slot base moved to an SGPR with v_readfirstlane two
# instructions before a global_load's `saddr` operand was read stale, which hung one run and
# faulted the next with an illegal memory access (commit 30ad87d).
DEVICE = os.path.join(ROOT, "msccl_amd", "csrc", "device")
MEM_INSN = re.compile(r"\b(global_|buffer_|flat_|scratch_|s_load|s_buffer_load|s_store|s_buffer_store|s_dcache)")
ALLOWED_INPUT = re.compile(r'^"[vin]"$')


def _asm_blocks(text):
    """(template, inputs) of every asm statement: the parenthesised body split at top-level colons."""
    out = []
    for m in re.finditer(r"\basm\s*(volatile\s*)?\(", text):
        i, depth, parts, cur, instr = m.end(), 1, [], [], False
        while i < len(text) and depth:
            ch = text[i]
            if ch == '"' and text[i - 1] != "\\":
                instr = not instr
            if not instr:
                if ch == "(":
                    depth += 1
                elif ch == ")":
                    depth -= 1
                    if depth == 0:
                        break
                elif ch == ":" and depth == 1:
                    parts.append("".join(cur))
                    cur = []
                    i += 1
                    continue
            cur.append(ch)
            i += 1
        parts.append("".join(cur))
        template = parts[0]
        inputs = parts[2] if len(parts) > 2 else ""
        out.append((template, re.findall(r'("[^"]*")\s*\(', inputs)))
    return out


def _bad_asm(text):
    return [(t.strip()[:60], c) for t, cons in _asm_blocks(text) if MEM_INSN.search(t)
            for c in cons if not ALLOWED_INPUT.match(c)]


def test_memory_asm_takes_vgpr_operands_only():
    srcs = glob.glob(os.path.join(DEVICE, "*.h")) + glob.glob(os.path.join(DEVICE, "*.hip"))
    assert srcs
    n = 0
    for f in srcs:
        text = open(f).read()
        n += sum(1 for t, _ in _asm_blocks(text) if MEM_INSN.search(t))
        assert _bad_asm(text) == [], f
    assert n >= 5   # the FIFO line polls (primitives.h: ldLines*) are found


def test_memory_asm_check_catches_an_sgpr_operand():
    ok = 'asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\\n\\ts_waitcnt vmcnt(0)" : "=&v"(x) : "v"(a) : "memory");'
    bad = ('asm volatile("global_load_dwordx4 %0, %1, %2 sc0 sc1\\n\\ts_waitcnt vmcnt(0)" : "=&v"(x) '
           ': "v"(off), "s"(base) : "memory");')
    reg = 'asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));'
    assert _bad_asm(ok) == [] and _bad_asm(reg) == []
    assert [c for _, c in _bad_asm(bad)] == ['"s"']


def test_every_type_object_holds_every_kernel_family():
    """Each per-type kernel object (build/obj/device/kernels_<type>.res) was compiled from the
    current kernels.h: it lists the general, small, fold, pair and two-phase kernels (a stale object once
    lacked the pair kernel and read RankWork at old offsets; init.cc also checks the layout stamp
    at run time)."""
    files = sorted(glob.glob(os.path.join(RES, "kernels_*.res")))
    files = [f for f in files if not re.search(r"kernels_(clock|probe)\.res$", f)]
    if not files:
        pytest.skip("no kernel resource reports (run __graft_entry__.build() first)")
    assert len(files) == 10, files
    for f in files:
        text = open(f).read()
        for fam in ("mscclKernel", "mscclSmallKernel", "mscclFoldKernel", "mscclPairKernel", "mscclTwoPhaseKernel"):
            assert re.search(r"Function Name: _ZN5msccl\d*%sI" % fam, text), (os.path.basename(f), fam)
