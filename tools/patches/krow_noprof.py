# timing knob: the profiler wave fills the profile ring once (the first LW columns) and then
# publishes "everything built": strips read a stale profile past that (results WRONG).  Prices
# the profiler's share of the CU (LDS traffic, issue slots of the SIMD it shares with strip 1).
a = "                flag_st(F + kFXo, qn > Cp ? kBig : qn);"
assert s.count(a) == 1
s = s.replace(a, "                if (qn >= kLW) qn = Cp + 1;\n" + a)
