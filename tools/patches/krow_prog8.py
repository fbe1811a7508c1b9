# K-rows variant: progress words read at step 8 of a block instead of step 14.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("            if (u == kBlk - 2)", "            if (u == 8)")
