# Halo reads awaited per quarter: the block-start asm waits for the first 16-byte read only
# (lgkmcnt(3)); steps 4, 8 and 12 wait for the next one with a count of the LDS ops known to be
# younger (the other halo reads + at least 2 ds_read2 of profile per row per 4 steps issued
# before that step; more younger ops only make the wait stricter).
a = """                "s_mov_b64 exec, %4\\n"
                "s_waitcnt lgkmcnt(0)"
                : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&s"(sv)"""
assert s.count(a) == 1
s = s.replace(a, """                "s_mov_b64 exec, %4\\n"
                "s_waitcnt lgkmcnt(3)"
                : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&s"(sv)""")
a = """            int nh[K];
            const int up = shr1z(H[K - 1]) + hc[u >> 2][u & 3];"""
assert s.count(a) == 1
s = s.replace(a, """            int nh[K];
            static_assert(K == 4 || K == 2, "halo wait counts assume K profile rows per step");
            if (u == 4) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(hc[1]) : "n"(2 + 2 * K) : "memory");
            if (u == 8) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(hc[2]) : "n"(1 + 4 * K > 15 ? 15 : 1 + 4 * K) : "memory");
            if (u == 12) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(hc[3]) : "n"(4 * K > 15 ? 15 : 4 * K) : "memory");
            const int up = shr1z(H[K - 1]) + hc[u >> 2][u & 3];""")
