# timing knob: the lane fill's step without profile reads and with one max instead of max3 (the
# output stores, hand-off and their pattern unchanged): prices how fast the full batch's stores
# drain when the compute between them is lighter.  Results WRONG.
a = "            for (int u = 0; u < kLBlk; ++u) qn[u] = lds_ld(qb + 4u * u);"
assert s.count(a) == 1
s = s.replace(a, "            for (int u = 0; u < kLBlk; ++u) qn[u] = (int)qb + u;")
a = "            int h = max(max(t1, up), hg);"
assert s.count(a) == 1
s = s.replace(a, "            int h = max(t1, up);")
