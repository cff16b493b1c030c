"""Print the memory/LDS/barrier skeleton of one kernel in a hipcc -save-temps .s file.
    python tools/isa_seq.py file.s name_substring"""
import re, sys
s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z\S+):', s, re.M)
name = [n for n in names if sys.argv[2] in n][0]
body = s.split(name + ':', 1)[1].split('.Lfunc_end', 1)[0]
seq = []
n = 0
for l in body.split('\n'):
    l = l.strip()
    if not l or l[0] in ';.' or l.endswith(':'):
        continue
    n += 1
    op = l.split()[0]
    if op.startswith('buffer_load'): seq.append('L')
    elif op.startswith('s_waitcnt'): seq.append('W(' + l.split(None, 1)[1] + ')')
    elif op.startswith('ds_read') or op.startswith('ds_load'): seq.append('r')
    elif op.startswith('ds_write') or op.startswith('ds_store'): seq.append('w')
    elif op == 's_barrier': seq.append('B')
    elif op.startswith('s_cbranch') or op == 's_branch': seq.append('J')
    elif op.startswith('global_load'): seq.append('G')
    elif op.startswith('global_store') or op.startswith('buffer_store'): seq.append('S')
print(name, n, 'instructions')
print(' '.join(seq))
m = re.search(re.escape(name) + r'.*?\.vgpr_count:\s+(\d+)', s[s.index('amdhsa.kernels'):], re.S)
