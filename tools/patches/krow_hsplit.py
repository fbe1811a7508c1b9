# The hand-off of a block in two halves: lane 63's values of steps 0..7 written after step 7 (inside
# the block, under the steps' latency), steps 8..15 at the block's end with the progress word: the
# block boundary carries 2 ds_write_b128 instead of 4.
a = """            lt[u] = H[K - 1];  // column t-64 of the lane's last row: ring element t"""
assert s.count(a) == 1
s = s.replace(a, a + """
            if (u == kBlk / 2 - 1)
            {
                const uint32_t eb = ring_out + 4u * (uint32_t)((kBlk * b) & (kRing - 1));
                uint64_t sv;
                asm volatile(
                    "s_mov_b64 %0, exec\\n"
                    "s_mov_b64 exec, %1\\n"
                    "ds_write_b128 %2, %3\\n"
                    "ds_write_b128 %2, %4 offset:16\\n"
                    "s_mov_b64 exec, %0"
                    : "=&s"(sv)
                    : "s"(1ull << 63), "v"(eb), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]})
                    : "memory");
            }""")
a = """            asm volatile(
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
                : "memory");"""
assert s.count(a) == 1
s = s.replace(a, """            asm volatile(
                "s_mov_b64 %0, exec\\n"
                "s_mov_b64 exec, %1\\n"
                "ds_write_b128 %2, %3 offset:32\\n"
                "ds_write_b128 %2, %4 offset:48\\n"
                "s_mov_b64 exec, %0"
                : "=&s"(sv)
                : "s"(1ull << 63), "v"(eb), "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]})
                : "memory");""")
