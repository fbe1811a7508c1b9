# NOT CORRECT in the score modes (profiles/r03_strip_h63.txt); kept as a record of the probe
# Strip kernel hand-off writes by lane 63 alone (exec mask set and restored inside one asm block,
# as the K-rows kernel does) instead of every lane writing its diagonal ring slot: only lane 63's
# slots are ever read (the next strip's halo and the drain).
a = """            lds_st4(ring_out + 16u * (uint32_t)(((t0 >> 2) - lane) & (kRing - 1)), int4v {Xd[0], Xd[1], Xd[2], Xd[3]});
            if constexpr (is_score_mode(MODE))
                lds_st4(ring2_out + 16u * (uint32_t)(((t0 >> 2) - lane) & (kRing - 1)), int4v {Fd[0], Fd[1], Fd[2], Fd[3]});"""
assert s.count(a) == 1
s = s.replace(a, """            {
                const uint32_t slot = 16u * (uint32_t)(((t0 >> 2) - lane) & (kRing - 1));
                uint64_t sv;
                if constexpr (is_score_mode(MODE))
                    asm volatile(
                        "s_mov_b64 %0, exec\\n"
                        "s_mov_b64 exec, %1\\n"
                        "ds_write_b128 %2, %3\\n"
                        "ds_write_b128 %4, %5\\n"
                        "s_mov_b64 exec, %0"
                        : "=&s"(sv)
                        : "s"(1ull << 63), "v"(ring_out + slot), "v"(int4v {Xd[0], Xd[1], Xd[2], Xd[3]}),
                          "v"(ring2_out + slot), "v"(int4v {Fd[0], Fd[1], Fd[2], Fd[3]})
                        : "memory");
                else
                    asm volatile(
                        "s_mov_b64 %0, exec\\n"
                        "s_mov_b64 exec, %1\\n"
                        "ds_write_b128 %2, %3\\n"
                        "s_mov_b64 exec, %0"
                        : "=&s"(sv)
                        : "s"(1ull << 63), "v"(ring_out + slot), "v"(int4v {Xd[0], Xd[1], Xd[2], Xd[3]})
                        : "memory");
            }""")
