"""Static check of the inline-asm LDS reads in a compiled kernel (hipcc -S output).

csrc/tail.hip issues its fragment reads as inline-asm ``ds_read_b128`` and waits for them with
explicit ``s_waitcnt lgkmcnt(N)``: the compiler believes an asm output register holds its value
as soon as the asm statement retires, while the hardware writes it when the read returns.  Any
instruction that reads or overwrites such a register before a wait retires the read is a race
(a register-allocator copy of a prefetched fragment, or reuse of a pending destination).

This walks the kernel's instruction stream in order (LDS operations complete in order; the
queue of pending reads is trimmed at every lgkmcnt wait), once through the function and once
more through every loop body entered with the state at its back edge, and reports every
access to a pending destination register.

    python tools/lds_async_check.py build/tail.s tail_kernelILi384ELb1E
"""
import re
import sys


def regs(tok):
    """v5 -> {v5}; v[4:7] -> {v4..v7}; a[0:3] -> {a0..a3}"""
    m = re.fullmatch(r"([va])(\d+)", tok)
    if m:
        return {tok}
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    return set()


def operands(line):
    body = line.split(";")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    return parts[0], [t.strip() for t in parts[1].split(",")]


def walk(lines, pending, report, tag):
    for no, raw in lines:
        op, ops = operands(raw)
        if not op or op.startswith((".", ";")) or op.endswith(":"):
            continue
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", raw)
            if m:
                while len(pending) > int(m.group(1)):
                    pending.pop(0)
            continue
        touched = set()
        for t in ops:
            touched |= regs(t.split()[0]) if t else set()
        for (pno, dst) in pending:
            hit = touched & dst
            if hit:
                report.append(f"{tag} line {no}: {raw.strip()}  touches {sorted(hit)[:4]} pending from line {pno}")
        if op.startswith("ds_read") or op.startswith("ds_load"):
            pending.append((no, regs(ops[0])))
        elif op.startswith("ds_") and not op.startswith("ds_write") and not op.startswith("ds_store"):
            pending.append((no, set()))                 # other LDS ops count toward lgkmcnt
        elif op.startswith("ds_write") or op.startswith("ds_store"):
            pending.append((no, set()))
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            pass                                       # SMEM: out of order, not tracked


def main(path, pat):
    text = open(path).read().split("\n")
    start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*" + pat + r"\S*:", l))
    end = next(i for i in range(start, len(text)) if text[i].startswith(".Lfunc_end"))
    lines = [(i + 1, text[i]) for i in range(start, end)]
    labels = {m.group(1): k for k, (_, l) in enumerate(lines) if (m := re.match(r"^(\.LBB\w+):", l))}
    report = []
    pending = []
    walk(lines, pending, report, "linear")
    for k, (_, l) in enumerate(lines):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            body = lines[labels[m.group(1)]:k + 1]
            st = []
            walk(body, st, [], "warm")                   # state at the back edge
            walk(body, st, report, f"loop {m.group(1)}")
    for r in report[:50]:
        print(r)
    print(f"{len(report)} hazard(s)")
    return 1 if report else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
