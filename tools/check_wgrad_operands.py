"""ISA check of k_wgrad_rect's staging loads (and of k_wgrad_dma's LDS-DMA loads) ("The k_wgrad_rect zeros"): compiles
csrc/x3mlp.hip for gfx950 and, in every k_wgrad_rect instantiation, collects the operand registers of the
full-step staging loads (the buffer_load_dword whose VGPR offset the kernel advances in place: that
VGPR, the SGPR resource, the SGPR offset if any) and lists every instruction from the first such load to the kernel's range-guard epilogue
that writes one of them.  The only writes allowed are the in-place v_add_u32 advances of the VGPR offsets
(the loads' own destinations never alias an operand) -- between a register's first use by a staging load and
the loop's last barrier.  Exit status 1 when any other write is found.

  python tools/check_wgrad_operands.py [-DDEFINE ...]
"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "marl-maze_amd", "csrc", "x3mlp.hip")


def regs(tok):
    m = re.fullmatch(r"([sv])(\d+)", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    m = re.fullmatch(r"([sv])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), k) for k in range(int(m.group(2)), int(m.group(3)) + 1)}
    return set()


NO_DST = ("s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop", "ds_write", "buffer_store", "global_store",
          "global_atomic", "s_cmp", "s_bitcmp", "s_endpgm", "s_setprio", "s_sleep", "v_cmpx", "s_sendmsg")


def dst(line):
    t = line.strip()
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        return None, set()
    op, _, args = t.partition(" ")
    if op.startswith(NO_DST) or (op.startswith("v_cmp_") and not op.endswith("_e64")) or \
            (op.startswith("buffer_load") and args.rstrip().endswith(" lds")):  # LDS-DMA: no register destination
        return op, set()
    return op, regs(args.split(",")[0].strip())


def main():
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "--cuda-device-only", "-S", "-I", os.path.join(REPO, "include"),
                        "-I", os.path.dirname(SRC), *defs, "-o", os.path.join(d, "k.s"), SRC], check=True,
                       stderr=subprocess.DEVNULL)
        asm = open(os.path.join(d, "k.s")).read().split("\n")
    bad = 0
    starts = [i for i, l in enumerate(asm) if re.match(r"^_ZN2mm2x3(12k_wgrad_rect|11k_wgrad_dma).*:", l)]
    for s0 in starts:
        name = asm[s0].split(":")[0]
        end = next(i for i in range(s0, len(asm)) if "s_endpgm" in asm[i])
        body = asm[s0:end]
        # the staging loads: their VGPR offset is one the kernel advances in place (v_add_u32 vX, vX, s..)
        pinned = {m.group(1) for m in (re.match(r"\s+v_add_u32 (v\d+), \1, s\d+$", l) for l in body) if m}
        first_use = {}  # operand register -> index of the first staging load reading it (outside the markers)
        inpart = False
        for i, l in enumerate(body):
            inpart = (inpart or ";;wg-partial-begin" in l) and ";;wg-partial-end" not in l
            if inpart:
                continue
            m = re.match(r"\s+buffer_load_dword (v\d+), (v\d+), (s\[\d+:\d+\]), (s\d+|0) offen", l)
            if m and m.group(2) in pinned:
                for r in regs(m.group(2)) | regs(m.group(3)) | regs(m.group(4)):
                    first_use.setdefault(r, i)
            # k_wgrad_dma's LDS-DMA loads (buffer_load_dwordx4 vOFF, s[rsrc], soff offen lds): every one
            m = re.match(r"\s+buffer_load_dwordx4 (v\d+), (s\[\d+:\d+\]), (s\d+|0) offen lds", l)
            if m:
                for r in regs(m.group(1)) | regs(m.group(2)) | regs(m.group(3)):
                    first_use.setdefault(r, i)
        # every staging load has landed by the loop's last barrier (its values were converted and stored before
        # it); hold_operands() keeps the operands live at least that far
        hold = max(i for i, l in enumerate(body) if "s_barrier" in l)
        hits = []
        skip = False  # inside the partial-step loads (the kernel's ;;wg-partial-begin / -end markers): nothing
        for i in range(len(body)):  # is in flight there, and their temporaries are waited for (vmcnt(0))
            if ";;wg-partial-begin" in body[i]:
                skip = True
            elif ";;wg-partial-end" in body[i]:
                skip = False
            if skip:
                continue
            op, w = dst(body[i])
            for r in w:
                if r in first_use and first_use[r] < i < hold and not (op == "v_add_u32" and len(w) == 1):
                    hits.append(body[i].strip())
                    break
        ops = first_use
        dem = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
        print(f"{dem[:60]:60s} operand regs {len(ops):3d}  foreign writes {len(hits)}")
        for h in hits[:8]:
            print("    ", h)
        bad += len(hits)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
