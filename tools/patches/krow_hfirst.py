# The next block's halo reads issued before this block's hand-off writes, in ONE asm block
# (halo reads, hand-off writes, progress write, then lgkmcnt(5): the reads are done, the writes
# may still run): the read latency no longer queues behind the writes.  One asm, because the
# compiler copies asm-written registers freely (a split issue/wait would copy stale halo values).
a = """        halo_load(b);
        const uint32_t pn = q_off(b + 1);"""
assert s.count(a) == 1
s = s.replace(a, """        if (b == 0 || hpend) halo_load(b);  // otherwise the halo came with the previous block's hand-off
        const uint32_t pn = q_off(b + 1);""")
a = """        handoff(b);
        if (CAP && cap)"""
assert s.count(a) == 1
s = s.replace(a, """        if (b + 1 < NB)
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            asm volatile("" ::"v"(rpin), "v"(rpco), "v"(rpxo), "v"(rsink));
            hpend = !ok(pin, pco, pxo, b + 1);
            if (hpend)
                handoff(b);  // publish first; the next block waits and reads its halo at its start
            else
                xfer(b);
        }
        else
            handoff(b);
        if (CAP && cap)""")
a = """        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            // every destination register"""
assert s.count(a) == 1
s = s.replace(a, """        if (b == 0 || hpend)  // otherwise checked at the previous block's end
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            // every destination register""")
a = """    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in mid-block, checked at the next block"""
assert s.count(a) == 1
s = s.replace(a, """    // block bb's hand-off with block bb+1's halo: lane 0 reads the halo, lane 63 writes its 16
    // values, all lanes write the progress words; only the reads are awaited
    auto xfer = [&](int bb) {
        const uint32_t hb = ring_in + 4u * (uint32_t)((kBlk * (bb + 1) + 64) & (kRing - 1));
        const uint32_t eb = ring_out + 4u * (uint32_t)((kBlk * bb) & (kRing - 1));
        const int2v fw = int2v {bb + 1 == NB ? kBig : kBlk * bb + kBlk, kBlk * bb + 64 + kBlk};
        uint64_t sv;
        asm volatile(
            "s_mov_b64 %4, exec\\n"
            "s_mov_b64 exec, 1\\n"
            "ds_read_b128 %0, %5\\n"
            "ds_read_b128 %1, %5 offset:16\\n"
            "ds_read_b128 %2, %5 offset:32\\n"
            "ds_read_b128 %3, %5 offset:48\\n"
            "s_mov_b64 exec, %6\\n"
            "ds_write_b128 %7, %8\\n"
            "ds_write_b128 %7, %9 offset:16\\n"
            "ds_write_b128 %7, %10 offset:32\\n"
            "ds_write_b128 %7, %11 offset:48\\n"
            "s_mov_b64 exec, %4\\n"
            "ds_write_b64 %12, %13\\n"
            "s_waitcnt lgkmcnt(5)"
            : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&s"(sv)
            : "v"(hb), "s"(1ull << 63), "v"(eb), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}),
              "v"(int4v {lt[4], lt[5], lt[6], lt[7]}), "v"(int4v {lt[8], lt[9], lt[10], lt[11]}),
              "v"(int4v {lt[12], lt[13], lt[14], lt[15]}), "v"(f_out), "v"(fw)
            : "memory");
    };
    bool hpend = false;  // the next block's check failed at this block's end: it waits and reads its halo itself
    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in mid-block, checked at the next block""")
