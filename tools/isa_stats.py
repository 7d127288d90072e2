"""Per-basic-block instruction counts of one kernel in a gfx950 assembly listing.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o k.s parquet-mr_amd/csrc/<file>.hip
  python3 tools/isa_stats.py k.s <kernel-name-substring> [--min N]

Prints the kernel's register / LDS / scratch figures and, for every basic block with at least
N instructions, its size and instruction mix (used to find the VALU-heavy loops)."""
import collections
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 20
    s = open(path).read()
    names = [n for n in re.findall(r"^(\S+):\s*; @", s, re.M) if pat in n]
    for name in names:
        a = s.index(name + ":")
        b = s.index(".Lfunc_end", a)
        body = s[a:b].split("\n")
        blocks, cur, label = [], [], name
        for ln in body[1:]:
            m = re.match(r"^(\.LBB\S+):", ln)
            if m:
                blocks.append((label, cur))
                label, cur = m.group(1), []
            elif ln.startswith("\t") and not ln.startswith("\t.") and not ln.startswith("\t;"):
                cur.append(ln.split()[0])
        blocks.append((label, cur))
        total = sum(len(c) for _, c in blocks)
        print(f"== {name}: {total} instructions, {len(blocks)} blocks")
        meta = s[b:b + 4000]
        for key in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size"):
            m = re.search(rf"\.{key}:\s+(\d+)", s[s.find(f".name:           {name}"):][:3000]) or re.search(rf"\.{key}:\s+(\d+)", meta)
            if m:
                print(f"   {key} = {m.group(1)}")
        for lab, ins in blocks:
            if len(ins) >= mn:
                c = collections.Counter(i.split("_")[0] for i in ins)
                print(f"   {lab:28s} {len(ins):5d}  " + " ".join(f"{k}:{v}" for k, v in c.most_common(8)))


if __name__ == "__main__":
    main()
