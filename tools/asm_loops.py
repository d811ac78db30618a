"""Spill report for a kernel in a hipcc -S dump: scratch ops inside each backward-branch loop.
python tools/asm_loops.py file.s <kernel-substring>"""
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2]
for name in [l.split(':')[0] for l in s.split('\n') if sub in l and l.startswith('_Z') and ': ;' in l]:
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    body = s[i:j].split('\n')
    labels = {l.split(':')[0]: k for k, l in enumerate(body) if l.startswith('.LBB')}
    tot = sum(1 for x in body if 'scratch_' in x)
    out = []
    for k, l in enumerate(body):
        if 's_branch' in l or 's_cbranch' in l:
            t = l.split()[-1]
            if t in labels and labels[t] < k:
                mf = sum(1 for x in body[labels[t]:k] if 'v_mfma' in x)
                if mf:
                    sc = sum(1 for x in body[labels[t]:k] if 'scratch_' in x)
                    out.append(f"mfma-loop len {k - labels[t]} mfma {mf} scratch {sc}")
    print(name[:90], 'scratch total', tot, '|', '; '.join(out))
