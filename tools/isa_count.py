#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S device assembly file:
  python tools/isa_count.py DEV.s MANGLED_NAME_PREFIX"""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
i = s.find("\n" + sys.argv[2])
i = s.find(":", i)
j = s.find(".Lfunc_end", i)
ins = [l.strip().split()[0] for l in s[i:j].split("\n")
       if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = Counter(ins)
print("total", len(ins), "valu", sum(v for k, v in c.items() if k.startswith("v_")),
      "salu", sum(v for k, v in c.items() if k.startswith("s_")),
      "vmem", sum(v for k, v in c.items() if k.startswith(("buffer_", "global_"))))
print(c.most_common(30))
