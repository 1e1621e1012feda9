"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (resource_usage.txt)."""
import re, sys, subprocess
txt = open(sys.argv[1] if len(sys.argv) > 1 else 'resource_usage.txt').read()
cur = None
rows = []
for line in txt.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip()
        except Exception:
            pass
        cur = {'name': name}
        rows.append(cur)
        continue
    for key in ('VGPRs', 'AGPRs', 'ScratchSize [bytes/lane]', 'Occupancy [waves/SIMD]', 'SGPRs'):
        m = re.search(re.escape(key) + r': (\d+)', line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    n = r['name'].replace('HIP_vector_type<float, 2u>', 'cf').replace('admm::', '')
    n = re.sub(r'\(.*', '', n)
    print(f"{n:45s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} scratch={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')}")
