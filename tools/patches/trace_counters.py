# nw_trace_dev.hip timing build: per-walk counters printed by thread 0 at the end (device printf):
# tiles copied from the band, tiles recomputed on entry, and s_memtime cycles spent in each and in
# the walk itself.  Diagnostics only.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a[:80]
    s = s.replace(a, b)
rep("""    long long n = 0;
""", """    long long n = 0;
    unsigned long long c_copy = 0, c_comp = 0, c_walk = 0, n_copy = 0, n_comp = 0;
""")
rep("""            if (slot >= 0)
            {""", """            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            if (slot >= 0)
            {
                ++n_copy;""")
rep("""            else
                tile_moves<DIRS_LDS>(a, iT, jT, iE, jE, sub, bnd, yraw, xraw, bprog, dirs, w, lane, first);
        }""", """            else
            {
                ++n_comp;
                tile_moves<DIRS_LDS>(a, iT, jT, iE, jE, sub, bnd, yraw, xraw, bprog, dirs, w, lane, first);
            }
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            if (slot >= 0) c_copy += t1 - t0; else c_comp += t1 - t0;
        }
        const unsigned long long tw0 = __builtin_amdgcn_s_memtime();""")
rep("""        __syncthreads();
        iT = state[0];""", """        __syncthreads();
        c_walk += __builtin_amdgcn_s_memtime() - tw0;
        iT = state[0];""")
rep("""    if (tid == 0) G(a.res)[0] = n;""", """    if (tid == 0) G(a.res)[0] = n;
    if (tid == 0)
        printf("trace counters: moves %lld copied %llu (%llu cyc) recomputed %llu (%llu cyc) walk %llu cyc\\n", n, n_copy,
               c_copy, n_comp, c_comp, c_walk);""")
