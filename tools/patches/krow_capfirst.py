# nw_krow.hip variant: the header-column capture runs before the block's hand-off (its VALU work
# overlaps the step-14 progress read instead of waiting behind the hand-off writes).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("""        handoff(b);
        if (CAP && cap)""", """        if (CAP && cap)""")
rep("""                hcolP += (size_t)(tBy + 1);
            }
        }
        return true;""", """                hcolP += (size_t)(tBy + 1);
            }
        }
        handoff(b);
        return true;""")
