"""Scan hipcc device assembly (hipcc --cuda-device-only -S) for a packed-FP32
VALU op (v_pk_*_f32) whose source VGPRs the NEXT instruction, an LDS or
vector-memory load, overwrites; prints per kernel the count and the first
pair (determinism audit).
usage: python tools/asm_war_scan.py file.s"""
import re,sys
s=open(sys.argv[1]).read().split('\n')
def regs(op):
    m=re.match(r'v\[(\d+):(\d+)\]',op)
    if m: return set(range(int(m.group(1)),int(m.group(2))+1))
    m=re.match(r'v(\d+)$',op)
    if m: return {int(m.group(1))}
    return set()
fn=None; hits={}
for i,l in enumerate(s):
    m=re.match(r'^(_Z\S+):',l)
    if m: fn=m.group(1)
    t=l.strip()
    if t.startswith('v_pk_') and '_f32' in t.split()[0]:
        ops=[o.strip() for o in t.split(None,1)[1].split(',')]
        src=set().union(*[regs(o.split()[0]) for o in ops[1:3]])
        # next real instruction
        j=i+1
        while j<len(s) and (not s[j].strip() or s[j].strip().startswith(';')): j+=1
        n=s[j].strip()
        if n.startswith('ds_read') or n.startswith('buffer_load') or n.startswith('global_load'):
            d=regs(n.split(None,1)[1].split(',')[0].strip())
            if d & src: hits.setdefault(fn,[]).append((i,t,n))
for f,h in hits.items(): print(f[:60], len(h), h[0])
