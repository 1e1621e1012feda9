"""Instruction mix of one kernel in the hipcc -S output (csrc/admm_capi.s).
usage: python tools/insmix.py <mangled-name-substring> [asm file]"""
import collections, re, sys
s = open(sys.argv[2] if len(sys.argv) > 2 else 'admm_capi.s').read()
m = re.search(r'^(\S*' + re.escape(sys.argv[1]) + r'\S*):', s, re.M)
start = m.end(); end = s.index('.Lfunc_end', start)
ops = collections.Counter()
loop_lines = 0
for line in s[start:end].splitlines():
    line = line.strip()
    if not line or line.startswith(('.', ';')) or line.endswith(':'):
        continue
    ops[line.split()[0]] += 1
print(m.group(1), 'total', sum(ops.values()))
cats = collections.Counter()
for k, v in ops.items():
    c = ('vmem' if k.startswith(('global_', 'buffer_')) else 'lds' if k.startswith('ds_') else
         'valu' if k.startswith('v_') else 'salu' if k.startswith('s_') else 'other')
    cats[c] += v
print(dict(cats))
for k, v in ops.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f'{k:28s}{v}')
