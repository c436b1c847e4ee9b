"""The wide-row GEMM (csrc/gemm256.hip) issues its MFMAs as inline asm (to pin each accumulator's
register class), so the compiler's hazard recognizer does not know they are MFMAs: an instruction
it places right after one — e.g. a register move re-homing an accumulator on the loop exit —
could read the accumulator before the MFMA has written it (seen once: 4 of 384 outputs of one
tile off by their last k16 step, only at 7 token groups).  This compiles the kernel to assembly
for gfx950 and checks that no instruction reads an MFMA's destination registers before the
drain (s_nop 7) or three further MFMAs.  The wide-row block tail (csrc/tailw.hip) is checked the
same way."""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "rag-snvbert_amd", "csrc")
# per-file flags of rag-snvbert_amd/Makefile (the scans must see the code that ships)
EXTRA = {"tailw.hip": ["-fno-slp-vectorize"]}


def _regs(tok):
    m = re.fullmatch(r"([av])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.fullmatch(r"([av])(\d+)", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def _reads(ins):
    ops = [o.strip() for o in ins.split(None, 1)[1].split(",")] if " " in ins else []
    src = ops[1:] if ops else []
    out = set()
    for o in src:
        out |= _regs(o.split()[0]) if o else set()
    return out


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
@pytest.mark.parametrize("src", ["gemm256.hip", "tailw.hip"])
def test_no_accumulator_read_inside_mfma_latency(tmp_path, src):
    """Also the wide-row block tail (csrc/tailw.hip), whose MFMAs are inline asm for the same reason."""
    SRC = os.path.join(CSRC, src)
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "g.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", *EXTRA.get(src, []), "-S", "--cuda-device-only",
                    SRC, "-o", str(out)], check=True, capture_output=True)
    lines = [ln.strip() for ln in out.read_text().split("\n")]
    ins = [ln for ln in lines if ln and not ln.startswith((";", ".", "_")) and not ln.endswith(":")]
    n_mfma = 0
    bad = []
    for i, t in enumerate(ins):
        if not t.startswith("v_mfma"):
            continue
        n_mfma += 1
        dst = _regs(t.split()[1].rstrip(","))
        later = 0
        for u in ins[i + 1:i + 80]:
            if u.startswith("s_nop 7") or u.startswith("s_endpgm"):
                break
            if u.startswith("v_mfma"):
                later += 1
                if later >= 3:
                    break
                continue
            if _reads(u) & dst:
                bad.append((t, u))
                break
    assert n_mfma > 1000
    assert not bad, bad[:5]


def _pending_reads(ins):
    """Reads of a register whose vector-memory load has not been retired by an s_waitcnt vmcnt yet
    (the waits counted in issue order, as the hardware does).  An inline-asm load hides its
    latency from the compiler, which may then copy the destination register (e.g. into an AGPR
    under register pressure) before the data lands."""
    pending, bad = [], []
    for i, t in enumerate(ins):
        op = t.split(" ")[0]
        m = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", t)
        if m:
            n = int(m.group(1))
            pending = pending[len(pending) - n:] if len(pending) > n else pending
            continue
        if op.startswith(("buffer_load", "global_load", "scratch_load")):
            pending.append(set() if " lds" in t else _regs(t.split(None, 1)[1].split(",")[0].strip()))
            continue
        if op.startswith(("buffer_store", "global_store", "scratch_store")):
            pending.append(set())
        if " " in t and op.startswith(("v_", "ds_write")):
            srcs = _reads(t) if op.startswith("v_") else set().union(*[_regs(o.strip().split()[0])
                                                                       for o in t.split(None, 1)[1].split(",") if o.strip()])
            if any(d & srcs for d in pending):
                bad.append((i, t))
    return bad


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_wide_tail_no_read_before_load_lands(tmp_path):
    """csrc/tailw.hip: no instruction reads a register still waiting for its load."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "t.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", *EXTRA["tailw.hip"], "-S",
                    "--cuda-device-only", os.path.join(CSRC, "tailw.hip"), "-o", str(out)], check=True,
                   capture_output=True)
    text = out.read_text().split("\n")
    for name in ("_ZN6snvrag12tailw_kernelILi0EEEvNS_6TwArgsE:", "_ZN6snvrag12projw_kernelENS_6PwArgsE:"):
        i0 = next(i for i, ln in enumerate(text) if ln.startswith(name))
        i1 = next(i for i in range(i0, len(text)) if text[i].strip().startswith(".Lfunc_end"))
        ins = [ln.strip() for ln in text[i0:i1]]
        ins = [ln for ln in ins if ln and not ln.startswith((";", ".", "_")) and not ln.endswith(":")]
        assert sum(t.startswith("v_mfma") for t in ins) > 250
        bad = _pending_reads(ins)
        assert not bad, (name, bad[:5])


def _valu_to_mfma(ins):
    """A VALU write (register copy, AGPR read, ...) of an MFMA source register fewer than 2 wait
    states before the inline-asm MFMA reading it: hipcc does not pad around asm it does not know is
    an MFMA, and the MFMA would read the stale value."""
    bad = []
    for i, t in enumerate(ins):
        if not t.startswith("v_mfma"):
            continue
        srcs = _reads(t)
        ws, k = 0, i - 1
        while k >= 0 and ws < 2:
            u = ins[k]
            if u.startswith("s_nop"):
                ws += int(u.split()[1]) + 1
            else:
                if u.startswith("v_") and not u.startswith("v_mfma") and " " in u and \
                        _regs(u.split(None, 1)[1].split(",")[0].strip()) & srcs:
                    bad.append((u, t))
                    break
                ws += 1
            k -= 1
    return bad


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_wide_tail_no_valu_write_before_mfma_operand(tmp_path):
    """csrc/tailw.hip: its FFN loop MFMAs carry no s_nop, so no VALU write may feed one directly."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "t.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", *EXTRA["tailw.hip"], "-S",
                    "--cuda-device-only", os.path.join(CSRC, "tailw.hip"), "-o", str(out)], check=True,
                   capture_output=True)
    text = out.read_text().split("\n")
    for name in ("_ZN6snvrag12tailw_kernelILi0EEEvNS_6TwArgsE:", "_ZN6snvrag12tailw_kernelILi1EEEvNS_6TwArgsE:",
                 "_ZN6snvrag12tailw_kernelILi8EEEvNS_6TwArgsE:", "_ZN6snvrag12tailw_kernelILi16EEEvNS_6TwArgsE:",
                 "_ZN6snvrag12projw_kernelENS_6PwArgsE:"):
        i0 = next(i for i, ln in enumerate(text) if ln.startswith(name))
        i1 = next(i for i in range(i0, len(text)) if text[i].strip().startswith(".Lfunc_end"))
        ins = [ln.strip() for ln in text[i0:i1]]
        ins = [ln for ln in ins if ln and not ln.startswith((";", ".", "_")) and not ln.endswith(":")]
        bad = _valu_to_mfma(ins)
        assert not bad, (name, bad[:5])


def _pending_writes(ins):
    """Writes to a register whose inline-asm vector-memory load has not been retired by an
    s_waitcnt vmcnt yet (the waits counted in issue order): the load lands later and overwrites
    the new value.  The compiler takes an asm load's destination as written at issue, so once the
    loaded value is dead (the K loop's last overrun loads) it may reuse the register at once."""
    pending, bad = [], []
    for i, t in enumerate(ins):
        op = t.split(" ")[0]
        m = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", t)
        if m:
            n = int(m.group(1))
            pending = pending[len(pending) - n:] if len(pending) > n else pending
            continue
        if op.startswith(("buffer_load", "global_load", "scratch_load")):
            pending.append(set() if " lds" in t else _regs(t.split(None, 1)[1].split(",")[0].strip()))
            continue
        if op.startswith(("buffer_store", "global_store", "scratch_store")):
            pending.append(set())
            continue
        if " " in t and (op.startswith(("v_", "ds_read")) and not op.startswith("v_accvgpr_write")):
            dst = _regs(t.split(None, 1)[1].split(",")[0].strip())
            if any(d & dst for d in pending):
                bad.append((i, t))
    return bad


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_gemm256_no_write_or_read_before_asm_load_lands(tmp_path):
    """csrc/gemm256.hip (the v2 kernel, every token-group count, plain and LayerNorm epilogues): from
    the K loop on (after the prologue's barrier), no instruction reads a register still waiting for
    its inline-asm W load, and none writes one — the r6 fault: the loop exit re-homed an accumulator
    into v[120:121] while the last K-step's overrun W load into v[120:123] was in flight."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "g.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "-S", "--cuda-device-only",
                    os.path.join(CSRC, "gemm256.hip"), "-o", str(out)], check=True, capture_output=True)
    text = out.read_text().split("\n")
    names = [f"_ZN6snvrag9g3_kernelILi{g}ELi0ELi{e}EEEvNS_6G2ArgsE:" for g in range(4, 9) for e in (0, 1)]
    for name in names:
        i0 = next(i for i, ln in enumerate(text) if ln.startswith(name))
        i1 = next(i for i in range(i0, len(text)) if text[i].strip().startswith(".Lfunc_end"))
        ins = [ln.strip() for ln in text[i0:i1]]
        ins = [ln for ln in ins if ln and not ln.startswith((";", ".", "_")) and not ln.endswith(":")]
        ins = ins[next(i for i, t in enumerate(ins) if t.startswith("s_barrier")):]
        assert sum(t.startswith("v_mfma") for t in ins) >= 48
        bad = _pending_writes(ins) + _pending_reads(ins)
        assert not bad, (name, bad[:5])

