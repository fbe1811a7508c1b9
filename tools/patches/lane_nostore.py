# timing knob: the lane fill's interior output stores skipped (values kept live by a never-true
# test), to price the compute side of a store-bound batch.  Results WRONG.
a = """                *(gptr<int4a>)(ub + xoff) = int4a {t[4 * k], t[4 * k + 1], t[4 * k + 2], t[4 * k + 3]};"""
assert s.count(a) == 1
s = s.replace(a, """                if ((t[4 * k] ^ t[4 * k + 1] ^ t[4 * k + 2] ^ t[4 * k + 3]) == 0x7fffeeee)
                    *(gptr<int4a>)(ub + xoff) = int4a {t[4 * k], t[4 * k + 1], t[4 * k + 2], t[4 * k + 3]};""")
