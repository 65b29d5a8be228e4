"""List the s_waitcnt vmcnt / s_barrier / MFMA / global memory lines of one
kernel in a -save-temps .s file, with the loop depth hipcc annotates, to see
where a kernel waits on outstanding loads.

  python3 tools/isa_waits.py file.s NAME_SUBSTRING [--all]
"""
import re
import sys

path, key = sys.argv[1], sys.argv[2]
s = open(path).read()
blks = [b for b in re.split(r'\n(?=_Z\S+:)', s) if key in b.split(':')[0]]
body = blks[0].split('.Lfunc_end')[0].split('\n')
depth = 0
pat = r'vmcnt|s_barrier|buffer_load|global_load|global_store|^\.LBB|s_cbranch|v_mfma' if '--all' in sys.argv \
    else r'vmcnt|s_barrier|buffer_load|global_load|^\.LBB.*Depth|v_mfma'
for i, l in enumerate(body):
    m = re.search(r'Depth=(\d+)', l)
    if m:
        depth = int(m.group(1))
    if re.search(pat, l):
        print("%5d d%d %s" % (i, depth, l.strip()[:100]))
