"""Static instruction histogram of one kernel in a -save-temps .s file:
MFMA / VALU / SALU / LDS / VMEM counts and the most frequent VALU opcodes.

  python3 tools/isa_hist.py file.s NAME_SUBSTRING
"""
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z\S*):', s, re.M)
for n in names:
    if sys.argv[2] not in n:
        continue
    body = s.split(n + ':')[1].split('.Lfunc_end')[0]
    lines = [l.strip() for l in body.split('\n')
             if l.strip() and not l.strip().startswith((';', '.'))]
    cats, h = {}, {}
    for l in lines:
        op = l.split()[0]
        c = ('mfma' if op.startswith('v_mfma') else 'valu' if op.startswith('v_') else
             'salu' if op.startswith('s_') else 'lds' if op.startswith('ds_') else
             'vmem' if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')) else 'other')
        cats[c] = cats.get(c, 0) + 1
        if c == 'valu':
            h[op] = h.get(op, 0) + 1
    print(n[:100])
    print("  ", cats)
    print("  ", sorted(h.items(), key=lambda x: -x[1])[:30])
