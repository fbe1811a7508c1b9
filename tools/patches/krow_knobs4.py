# K-rows timing knobs (results WRONG), chosen by KNOBS (comma list): noprof (next block's profile
# = this block's, no LDS reads), nohalo (no halo reads), nohand (no hand-off ring writes; progress
# words kept), nocap (no header-column capture), halfprof (rows K/2.. keep their profile: 8 reads per block).  Prices each component of a block.
import os
knobs = set(os.environ.get("KNOBS", "").split(","))
def rep(a, b, n=1):
    global s
    assert s.count(a) >= n, (a, s.count(a))
    s = s.replace(a, b, 1)
if "noprof" in knobs:
    rep("for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);", "for (int k = 0; k < K; ++k) qn[k][u] = qc[k][u];")
if "halfprof" in knobs:
    rep("for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);", "for (int k = 0; k < K; ++k) qn[k][u] = (k < K / 2) ? lds_ld(qrow[k] + pn + 4u * u) : qc[k][u];")
if "qtail" in knobs:
    # the reads of rows K/2.. only every other block (half the read instructions on average)
    rep("for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);", "for (int k = 0; k < K; ++k) qn[k][u] = (k < K / 2 || (b & 2)) ? lds_ld(qrow[k] + pn + 4u * u) : qc[k][u];")
if "nohalo" in knobs:
    rep('''                "s_mov_b64 %4, exec\\n"
                "s_mov_b64 exec, 1\\n"
                "ds_read_b128 %0, %5\\n"
                "ds_read_b128 %1, %5 offset:16\\n"
                "ds_read_b128 %2, %5 offset:32\\n"
                "ds_read_b128 %3, %5 offset:48\\n"
                "s_mov_b64 exec, %4\\n"
                "s_waitcnt lgkmcnt(0)"''', '''                "s_mov_b64 %4, exec\\n"''')
if "nohand" in knobs:
    rep('''                "s_mov_b64 %0, exec\\n"
                "s_mov_b64 exec, %1\\n"
                "ds_write_b128 %2, %3\\n"
                "ds_write_b128 %2, %4 offset:16\\n"
                "ds_write_b128 %2, %5 offset:32\\n"
                "ds_write_b128 %2, %6 offset:48\\n"
                "s_mov_b64 exec, %0"''', '''                "s_mov_b64 %0, exec\\n"''')
if "nocap" in knobs:
    rep("if (CAP && cap)\n", "if (CAP && cap && a.R < 0)\n")
