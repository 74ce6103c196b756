"""Summarise per-layer cycle traces printed by an SGUFP_TRACE build (last relax call)."""
import re
import statistics as st
import sys

rows = [tuple(map(int, re.findall(r'=(\d+)', l))) for l in open(sys.argv[1]) if l.startswith('L ')]
n = len(rows) // 4
rows = rows[-n:]
ex = [r for r in rows if r[2] == 0]
mg = [r for r in rows if r[2] > 0]
print("layers", len(rows), "exact", len(ex), "merged", len(mg), "total cyc", sum(r[4] for r in rows))
print("exact cyc mean %.0f median %.0f mean n %.1f" % (st.mean(r[4] for r in ex), st.median(r[4] for r in ex), st.mean(r[1] for r in ex)))
print("merged cyc mean %.0f median %.0f mean acnt %.1f" % (st.mean(r[4] for r in mg), st.median(r[4] for r in mg), st.mean(r[2] for r in mg)))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(r)
