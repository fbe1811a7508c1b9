# scheduling-group barriers over the block's steps: (8 VALU, 2 DS read) x 8, then the rest
# (guides the compiler's interleaving of the profile reads with the step chain)
a = """        // the block's hand-off at its end (the next strip sees it a block earlier than when it is"""
assert s.count(a) == 1
s = s.replace(a, """#pragma unroll
        for (int i = 0; i < 8; ++i)
        {
            __builtin_amdgcn_sched_group_barrier(0x2, 8, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
""" + a)
