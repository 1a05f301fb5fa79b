"""Basic-block census of one loop in a hipcc -S listing: instruction mix per block, so the hot path
can be told apart from rarely taken blocks.  usage: isa_blocks.py f.s kernel-substr loop-label"""
import re
import sys
from collections import Counter

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_loops import kind  # noqa: E402

src = open(sys.argv[1]).read().splitlines()
want, lab = sys.argv[2], sys.argv[3]
start = [i for i, l in enumerate(src) if l.startswith("_Z") and want in l.split(":")[0] and ":" in l][0]
body = src[start:]
i0 = [i for i, l in enumerate(body) if l.startswith(lab + ":")][0]
i1 = [i for i, l in enumerate(body) if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\s*$", l.strip())][-1]
blk, cnt, tot = lab, Counter(), Counter()
for l in body[i0:i1 + 1]:
    m = re.match(r"^(\.LBB[0-9_]+|; %bb\.[0-9]+):", l)
    if m:
        if cnt:
            print(f"{blk:14s} {sum(cnt.values()):5d} {dict(cnt)}")
        blk, cnt = m.group(1), Counter()
        continue
    t = l.split(";")[0].strip()
    if not t or t.startswith("."):
        continue
    cnt[kind(t.split()[0])] += 1
    tot[kind(t.split()[0])] += 1
print(f"{blk:14s} {sum(cnt.values()):5d} {dict(cnt)}")
print("total", sum(tot.values()), dict(tot))
