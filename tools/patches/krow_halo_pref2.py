# nw_krow.hip variant: the halo of block b+1 is read in the hand-off asm block at the end of block
# b (before the hand-off writes, after the step-14 progress read that validates it; LDS executes
# a wave's operations in order), and awaited there with the writes; block b+1 uses it when its
# check passes on those words and re-reads it just in time otherwise.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)

rep("""    int4v hc[kHalo];
#pragma unroll
    for (int j = 0; j < kHalo; ++j) hc[j] = int4v {0, 0, 0, 0};
    auto halo_load = [&](int b) {""", """    int4v hA[kHalo], hB[kHalo];
#pragma unroll
    for (int j = 0; j < kHalo; ++j) hA[j] = hB[j] = int4v {0, 0, 0, 0};
    auto halo_load = [&](int b, int4v (&hc)[kHalo]) {""")
rep("""    auto handoff = [&](int bb) {
        // lane 63 alone (exec set and restored inside the asm)
        const uint32_t eb = ring_out + 4u * (uint32_t)((kBlk * bb) & (kRing - 1));
        uint64_t sv;
        asm volatile(
            "s_mov_b64 %0, exec\\n"
            "s_mov_b64 exec, %1\\n"
            "ds_write_b128 %2, %3\\n"
            "ds_write_b128 %2, %4 offset:16\\n"
            "ds_write_b128 %2, %5 offset:32\\n"
            "ds_write_b128 %2, %6 offset:48\\n"
            "s_mov_b64 exec, %0"
            : "=&s"(sv)
            : "s"(1ull << 63), "v"(eb), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]}),
              "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]})
            : "memory");""", """    auto handoff = [&](int bb, int4v (&hn)[kHalo]) {
        // lane 0: block bb+1's halo (speculative); lane 63: the hand-off; exec set and restored
        // inside the asm, which awaits both
        const uint32_t eb = ring_out + 4u * (uint32_t)((kBlk * bb) & (kRing - 1));
        const uint32_t hb = ring_in + 4u * (uint32_t)((kBlk * (bb + 1) + 64) & (kRing - 1));
        uint64_t sv;
        asm volatile(
            "s_mov_b64 %4, exec\\n"
            "s_mov_b64 exec, 1\\n"
            "ds_read_b128 %0, %7\\n"
            "ds_read_b128 %1, %7 offset:16\\n"
            "ds_read_b128 %2, %7 offset:32\\n"
            "ds_read_b128 %3, %7 offset:48\\n"
            "s_mov_b64 exec, %5\\n"
            "ds_write_b128 %6, %8\\n"
            "ds_write_b128 %6, %9 offset:16\\n"
            "ds_write_b128 %6, %10 offset:32\\n"
            "ds_write_b128 %6, %11 offset:48\\n"
            "s_mov_b64 exec, %4"
            : "+v"(hn[0]), "+v"(hn[1]), "+v"(hn[2]), "+v"(hn[3]), "=&s"(sv)
            : "s"(1ull << 63), "v"(eb), "v"(hb), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]}),
              "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]})
            : "memory");""")
rep("""    auto block = [&](int b, int (&qc)[K][8], int (&qn)[K][8], auto rampT, bool cap) {""",
    """    auto block = [&](int b, int (&qc)[K][8], int (&qn)[K][8], int4v (&hc)[kHalo], int4v (&hn)[kHalo], auto rampT, bool cap) {""")
rep("""            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        halo_load(b);""", """            // ok: hc was read at the end of block b-1, behind the words just checked
            if (!ok(pin, pco, pxo, b))
            {
                if (!spin(b)) return false;
                halo_load(b, hc);
            }
        }""")
rep("""        handoff(b);
        if (CAP && cap)""", """        handoff(b, hn);
        if (CAP && cap)""")
rep("""                hcolP += (size_t)(tBy + 1);
            }
        }
        return true;""", """                hcolP += (size_t)(tBy + 1);
            }
        }
        // the speculative halo reads, awaited after the capture (its VALU work hides them)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(hn[0]), "+v"(hn[1]), "+v"(hn[2]), "+v"(hn[3])::"memory");
        return true;""")
rep("""        if (!block(b, qA, qB, T(), false)) return;
        if (!block(b + 1, qB, qA, T(), false)) return;""", """        if (!block(b, qA, qB, hA, hB, T(), false)) return;
        if (!block(b + 1, qB, qA, hB, hA, T(), false)) return;""")
rep("""        if (!block(b, qA, qB, F(), advance(b))) return;""", """        if (!block(b, qA, qB, hA, hB, F(), advance(b))) return;""")
rep("""        if (!block(b + 1, qB, qA, F(), advance(b + 1))) return;""", """        if (!block(b + 1, qB, qA, hB, hA, F(), advance(b + 1))) return;""")
