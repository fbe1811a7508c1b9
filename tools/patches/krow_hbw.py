# K-rows variant: the next block's progress check and halo reads are issued at the end of a block,
# BEFORE its hand-off writes, so waiting for the halo (at the next block's start, lgkmcnt(5): the 4
# hand-off writes and the progress word write are younger) does not wait for those writes (a wave's
# LDS operations complete in order).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a, s.count(a))
    s = s.replace(a, b)
# split halo load: issue (no wait) and wait (counted)
rep("""    auto halo_load = [&](int b) {""", """    auto halo_issue = [&](int b) {
        const uint32_t hb = ring_in + 4u * (uint32_t)((kBlk * b + 64) & (kRing - 1));
        uint64_t sv;
        asm volatile(
            "s_mov_b64 %4, exec\\n"
            "s_mov_b64 exec, 1\\n"
            "ds_read_b128 %0, %5\\n"
            "ds_read_b128 %1, %5 offset:16\\n"
            "ds_read_b128 %2, %5 offset:32\\n"
            "ds_read_b128 %3, %5 offset:48\\n"
            "s_mov_b64 exec, %4"
            : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&s"(sv)
            : "v"(hb)
            : "memory");
    };
    // the halo reads were followed by the 4 hand-off writes and the progress-word write
    auto halo_wait = [&]() {
        asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3])::"memory");
    };
    auto halo_load = [&](int b) {""")
rep("""            asm volatile("" ::"v"(rpin), "v"(rpco), "v"(rpxo), "v"(rsink));
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        halo_load(b);
        const uint32_t pn = q_off(b + 1);""", """            asm volatile("" ::"v"(rpin), "v"(rpco), "v"(rpxo), "v"(rsink));
            (void)pin; (void)pco; (void)pxo;
        }
        halo_wait();
        const uint32_t pn = q_off(b + 1);""")
rep("""        // the block's hand-off at its end (the next strip sees it a block earlier than when it is
        // written behind the next block's halo reads: measured 1 % faster at 100k, slightly slower
        // per block)
        handoff(b);""", """        // the next block's check and halo reads, then this block's hand-off writes (behind them in
        // the wave's LDS queue, so the halo wait does not include the writes)
        if (b + 1 < NB)
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            asm volatile("" ::"v"(rpin), "v"(rpco), "v"(rpxo), "v"(rsink));
            if (!ok(pin, pco, pxo, b + 1) && !spin(b + 1)) return false;
            halo_issue(b + 1);
        }
        handoff(b);""")
# the first block: issue its halo before the loop (after the initial spin) and a dummy 5-op gap
rep("""        if (!spin(-1)) return;""", """        if (!spin(-1)) return;
        if (!spin(0)) return;
        halo_load(0);
        halo_issue(0);  // re-issued so that block 0's halo_wait (lgkmcnt(5)) covers it
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3])::"memory");""")
