"""Flow-sensitive check of gfx950 kernel assembly: every SGPR a memory
instruction takes its address from (s_load / s_buffer_load base, global saddr,
buffer resource and soffset) must be written on EVERY path from the kernel
entry to it.

Why (DESIGN.md 4.2a, round-5 fault): the fused k_seg_combine of commit 4cd7616
read gridDim.x with `s_load_dword s26, s[48:49], 0x0` at the k_crc_any body's
entry.  The IR was sound (a phi of two llvm.amdgcn.implicitarg.ptr calls), but
the backend defined s[48:49] only on the k_crc_grp path; the plain-fallback
path reached the load with the pair marked `; implicit-def: $sgpr48_sgpr49`
(undefined), i.e. whatever the SIMD's previous wave left there -> an illegal
address on some boxes, a wrong grid size on others.

Usage: python tools/isa_sgpr_defs.py FILE.s [...]   (prints findings; rc 1 if any)
Library: check_text(asm_text) -> {kernel: [(line_no, instruction, undefined_sgprs)]}
"""
import re
import sys

_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
_BB_COMMENT = re.compile(r"^; %bb\.\d+:")
_SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
# scalar instructions without a scalar destination (the kernels here issue no
# scalar memory writes at all, so none are listed)
_NO_SDST = (
    "s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_endpgm", "s_sleep",
    "s_setprio", "s_sendmsg", "s_trap", "s_setreg", "s_set_gpr_idx", "s_icache", "s_wait", "s_ttrace",
    "s_denorm", "s_round",
)


def _regs(tok):
    out = set()
    for m in _SREG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _split_ops(rest):
    rest = rest.split(";")[0]
    return [o.strip() for o in rest.split(",")] if rest.strip() else []


def _writes(mn, ops):
    """SGPRs an instruction writes (its scalar destinations)."""
    if not ops:
        return set()
    if mn.startswith("s_"):
        if mn.startswith(_NO_SDST):
            return set()
        return _regs(ops[0])
    if mn.startswith("v_"):
        w = set()
        if mn.startswith(("v_readfirstlane", "v_readlane", "v_cmp", "v_cmpx")) or mn.endswith("_e64") and \
                mn.startswith("v_cmp"):
            w |= _regs(ops[0])
        if mn.startswith(("v_add_co", "v_sub_co", "v_subrev_co", "v_addc_co", "v_subb_co", "v_subbrev_co",
                          "v_mad_u64_u32", "v_mad_i64_i32", "v_div_scale")) and len(ops) > 1:
            w |= _regs(ops[1])
        return w
    return set()


def _address_sgprs(mn, ops):
    """SGPRs a memory instruction forms its address / resource from."""
    if mn.startswith(("s_load", "s_buffer_load")):
        return _regs(ops[1]) if len(ops) > 1 else set()
    if mn.startswith(("global_", "scratch_")):
        return set().union(*[_regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
    if mn.startswith("buffer_"):
        # buffer_load v, voff, s[rsrc], soffset ...
        return set().union(*[_regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
    return set()


def _entry_sgprs(meta):
    n = 0
    m = re.search(r"\.amdhsa_user_sgpr_count (\d+)", meta)
    if m:
        n = int(m.group(1))
    for k in ("workgroup_id_x", "workgroup_id_y", "workgroup_id_z", "workgroup_info",
              "private_segment_wavefront_offset"):
        m = re.search(rf"\.amdhsa_system_sgpr_{k} (\d+)", meta)
        if m and int(m.group(1)):
            n += 1
    return set(range(n))


def check_body(lines, entry):
    """lines: the kernel's assembly lines; entry: SGPRs defined at launch."""
    # basic blocks: split at labels, '; %bb.N:' markers and after every branch
    blocks, labels = [], {}
    cur = []

    def close():
        nonlocal cur
        if cur:
            blocks.append(cur)
        cur = []

    for no, raw in lines:
        s = raw.strip()
        m = _LABEL.match(s)
        if m or _BB_COMMENT.match(s):
            close()
            if m:
                labels[m.group(1)] = len(blocks)
            cur.append((no, s))
            continue
        cur.append((no, s))
        if s.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            close()
    close()
    succ = []
    for i, b in enumerate(blocks):
        last = b[-1][1]
        mn = last.split()[0] if last else ""
        t = []
        if mn.startswith(("s_branch", "s_cbranch")):
            tgt = last.split()[1]
            if tgt in labels:
                t.append(labels[tgt])
            if mn.startswith("s_cbranch") and i + 1 < len(blocks):
                t.append(i + 1)
        elif mn.startswith(("s_endpgm", "s_setpc")):
            pass
        elif i + 1 < len(blocks):
            t.append(i + 1)
        succ.append(t)
    pred = [[] for _ in blocks]
    for i, t in enumerate(succ):
        for j in t:
            pred[j].append(i)
    ALL = set(range(112))
    din = [set(ALL) for _ in blocks]
    if blocks:
        din[0] = set(entry)

    def transfer(i, state, report=None):
        d = set(state)
        for no, s in blocks[i]:
            if s.startswith(";"):
                m = re.search(r"implicit-def: (.*)", s)
                if m:
                    for r in re.findall(r"\$sgpr(\d+)", m.group(1)):
                        d.discard(int(r))
                continue
            if not s or s.startswith(".") or s.endswith(":"):
                continue
            parts = s.split(None, 1)
            mn = parts[0]
            ops = _split_ops(parts[1]) if len(parts) > 1 else []
            if report is not None:
                need = _address_sgprs(mn, ops)
                miss = need - d
                if miss:
                    report.append((no, s, sorted(miss)))
            d |= _writes(mn, ops)
        return d

    changed = True
    dout = [None] * len(blocks)
    while changed:
        changed = False
        for i in range(len(blocks)):
            if i:
                ins = [dout[p] for p in pred[i] if dout[p] is not None]
                new = set.intersection(*ins) if ins else set(ALL)
                if new != din[i]:
                    din[i] = new
            o = transfer(i, din[i])
            if o != dout[i]:
                dout[i] = o
                changed = True
    report = []
    for i in range(len(blocks)):
        # blocks no path reaches (din == ALL with no preds) are not checked
        if i and not pred[i]:
            continue
        transfer(i, din[i], report)
    return report


def check_text(text):
    out = {}
    metas = {m.group(1): m.group(2) for m in
             re.finditer(r"^\t\.amdhsa_kernel (\S+)\n(.*?)\t\.end_amdhsa_kernel", text, re.S | re.M)}
    all_lines = text.split("\n")
    for name, meta in metas.items():
        start = text.index(f"\n{name}:")
        first = text.count("\n", 0, start) + 2
        end = text.index(f"\t.amdhsa_kernel {name}\n")
        last = text.count("\n", 0, end)
        lines = [(k + 1, all_lines[k]) for k in range(first - 1, last)]
        rep = check_body(lines, _entry_sgprs(meta))
        if rep:
            out[name] = rep
    return out


def main(paths):
    bad = 0
    for p in paths:
        res = check_text(open(p).read())
        for k, rep in res.items():
            bad += 1
            print(f"{p}: {k}")
            for no, s, miss in rep[:8]:
                print(f"  line {no}: {s}    undefined on some path: s{miss}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
