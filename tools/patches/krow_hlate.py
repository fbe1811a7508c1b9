# K-rows variant: block b's hand-off (lane 63's ring writes + the progress word) issued at the start
# of block b+1, right after that block's halo wait, instead of at the end of block b: the next
# block's progress check and halo read then no longer wait for the four ds_write_b128 to drain
# through the wave's in-order LDS queue.  The first call (b = 0) writes ring slots no reader has
# reached and publishes {0, 64} (nothing).  The strip's last block is handed off after the loop.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a, s.count(a))
    s = s.replace(a, b)
rep("""        halo_load(b);
        const uint32_t pn = q_off(b + 1);""", """        halo_load(b);
        handoff(b - 1);
        const uint32_t pn = q_off(b + 1);""")
rep("""        handoff(b);
        if (CAP && cap)""", """        if (CAP && cap)""")
rep("""    if (pt)
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        flag_st(L.flags + kFCap + 4u * (uint32_t)w, kBig);""", """    handoff(NB - 1);
    if (pt)
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        flag_st(L.flags + kFCap + 4u * (uint32_t)w, kBig);""")
