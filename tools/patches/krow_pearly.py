# The next block's progress check evaluated at the end of this block, before its hand-off
# writes: the readfirstlane of the words (read at step 14) then waits for that read only, not
# for the hand-off writes the compiler cannot see; a failed check still spins at the next
# block's start (after the hand-off is published).
a = """        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            // every destination register"""
assert s.count(a) == 1
s = s.replace(a, """        if (b == 0)
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            nready = !ok(pin, pco, pxo, b);
        }
        if (nready && !spin(b)) return false;
        if (false)
        {
            const int pin = 0, pco = 0, pxo = 0;
            // every destination register""")
a = """        handoff(b);
        if (CAP && cap)"""
assert s.count(a) == 1
s = s.replace(a, """        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            asm volatile("" ::"v"(rpin), "v"(rpco), "v"(rpxo), "v"(rsink));
            nready = !ok(pin, pco, pxo, b + 1);
        }
        handoff(b);
        if (CAP && cap)""")
a = """    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in mid-block, checked at the next block"""
assert s.count(a) == 1
s = s.replace(a, """    bool nready = false;               // the next block's progress check failed (evaluated at this block's end)
    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in mid-block, checked at the next block""")
