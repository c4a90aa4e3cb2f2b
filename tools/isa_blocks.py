"""Basic blocks of one kernel in a device .s file (tools/isa.sh), with
instruction counts by class and the back edges (loops):
    python tools/isa_blocks.py FILE.s 'geo_render_kernelILi0ELi0E' [--print BLOCK...]"""
import re
import sys


def kernel_lines(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*%s\w*:" % sym, l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def blocks(lines):
    out, cur, name = [], [], "entry"
    for l in lines[1:]:
        s = l.split(";")[0].strip()
        m = re.match(r"^(\.LBB\w+):", s)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        if not s or s.startswith("."):
            continue
        cur.append(s)
    out.append((name, cur))
    return out


def klass(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    show = sys.argv[sys.argv.index("--print") + 1:] if "--print" in sys.argv else []
    bl = blocks(kernel_lines(path, sym))
    idx = {n: i for i, (n, _) in enumerate(bl)}
    tot = {}
    for i, (n, ins) in enumerate(bl):
        c = {}
        for x in ins:
            k = klass(x)
            c[k] = c.get(k, 0) + 1
            tot[k] = tot.get(k, 0) + 1
        br = [x for x in ins if x.startswith("s_cbranch") or x.startswith("s_branch")]
        back = [x.split()[-1] for x in br if x.split()[-1] in idx and idx[x.split()[-1]] <= i]
        print(f"{i:3d} {n:14s} valu {c.get('valu', 0):4d} salu {c.get('salu', 0):3d} vmem {c.get('vmem', 0):2d}"
              + (f"  back-> {back}" if back else "") + (f"  br {[x.split()[0] + ' ' + x.split()[-1] for x in br]}" if br else ""))
    print("total", tot)
    for n in show:
        print(f"--- {n}")
        for x in bl[idx[n]][1]:
            print("   ", x)


if __name__ == "__main__":
    main()
