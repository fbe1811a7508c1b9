# K-rows variant: progress words read at step 12 instead of 14.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a, s.count(a))
    s = s.replace(a, b)
rep("            if (u == kBlk - 2)", "            if (u == kBlk - 4)")
