exec(open('tools/patches/krow_qspread.py').read())
exec(open('tools/patches/krow_prog12.py').read())
