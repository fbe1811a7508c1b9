# K-rows variant: the block's progress words and its halo read together at block start (one LDS
# round trip: the words are read first, so halo values read behind a word that shows them published
# are the new ones), instead of a progress read at step 14 checked at block start plus the halo read.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("""    // profile dwords of block b: columns 16b - lane .. +15 are dwords 8b - lane/2 .. +7 of copy""",
"""    // block b's progress words and halo in one round trip, spinning (both re-read) until the block
    // may start: the halo reads follow the word read in the wave's in-order LDS queue, so values
    // read behind a word that shows them published are the new ones
    auto halo_prog = [&](int b) {
        const uint32_t hb = ring_in + 4u * (uint32_t)((kBlk * b + 64) & (kRing - 1));
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (int it = 1;; ++it)
        {
            int4v pr;
            uint64_t sv;
            asm volatile(
                "s_mov_b64 %5, exec\\n"
                "s_mov_b64 exec, 1\\n"
                "ds_read2_b64 %4, %7 offset1:2\\n"
                "ds_read_b128 %0, %6\\n"
                "ds_read_b128 %1, %6 offset:16\\n"
                "ds_read_b128 %2, %6 offset:32\\n"
                "ds_read_b128 %3, %6 offset:48\\n"
                "s_mov_b64 exec, %5\\n"
                "s_waitcnt lgkmcnt(0)"
                : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&v"(pr), "=&s"(sv)
                : "v"(hb), "v"(f_in)
                : "memory");
            const int pin = __builtin_amdgcn_readfirstlane(pr.x), pco = __builtin_amdgcn_readfirstlane(pr.w);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(pr.y) : 0;
            if (ok(pin, pco, pxo, b)) return true;
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || ((it & 31) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return false;
            }
        }
    };
    // profile dwords of block b: columns 16b - lane .. +15 are dwords 8b - lane/2 .. +7 of copy""")
rep("""        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        halo_load(b);""", """        if (!halo_prog(b)) return false;""")
rep("""            if (u == kBlk - 2)
            {
                // slot w-1 {prog[w], cons[w-1] | xo} and slot w+1 {prog[w+2], cons[w+1]}: one
                // ds_read2_b64 (plain loads, kept in place by the memory clobbers around them)
                asm volatile("" ::: "memory");
                const int2v lo = *(const int2v*)(krsm + f_in), hi = *(const int2v*)(krsm + f_in + 16u);
                asm volatile("" ::: "memory");
                rpin = lo.x;
                rpxo = lo.y;
                rpco = hi.y;
            }
""", "")
