"""Summarise -Rpass-analysis=kernel-resource-usage remarks (tools/ru.sh)."""
import re
import sys

cur, vals = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur, vals = m.group(1), {}
        continue
    for key, pat in (("v", r"VGPRs: (\d+)"), ("s", r"ScratchSize \[bytes/lane\]: (\d+)"), ("o", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("l", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur:
            vals[key] = m.group(1)
    if cur and "l" in vals:
        if "k_body" in cur or "k_refresh" in cur:
            name = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", cur)[:40]
            print("%-42s vgpr %4s scratch %4s occ %s lds %6s" % (name, vals["v"], vals["s"], vals["o"], vals["l"]))
        cur = None
