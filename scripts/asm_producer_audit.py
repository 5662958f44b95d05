"""Resident-solver diagnostics (DESIGN_HISTORY §4i): DPP inline-asm results consumed by
compiler-emitted instructions within the hazard window, by consumer kind and wait
states (clang -S output of scripts/serve_variant_src.py)."""
import re, sys
lines = open(sys.argv[1]).read().split("\n")
def vregs(ops):
    out=[]
    for t in ops:
        t=t.strip().lstrip("-|")
        m=re.match(r"v\[(\d+):(\d+)\]",t)
        if m: out.append((int(m.group(1)),int(m.group(2)))); continue
        m=re.match(r"v(\d+)$",t)
        if m: out.append((int(m.group(1)),)*2)
    return out
insns=[]; inasm=False
for i,l in enumerate(lines):
    s=l.strip()
    if s.startswith(";;#ASMSTART"): inasm=True; continue
    if s.startswith(";;#ASMEND"): inasm=False; continue
    if not s or s.startswith(";") or s.startswith("."): 
        if re.match(r"^\.LBB",s): insns.append(("LABEL",[],i,False,s))
        continue
    if s.endswith(":"): insns.append(("LABEL",[],i,False,s)); continue
    parts=s.split(None,1); mn=parts[0]; ops=parts[1].split(",") if len(parts)>1 else []
    ops=[o.split()[0] if o.strip() else o for o in ops]
    insns.append((mn,vregs(ops),i,inasm,s))
from collections import Counter
hits=Counter(); ex={}
for k,(mn,vr,i,asm,s) in enumerate(insns):
    if not (asm and "_dpp" in mn) or not vr: continue
    d=vr[0]; ws=0
    for j in range(k+1,min(k+8,len(insns))):
        mn2,vr2,i2,asm2,s2=insns[j]
        if mn2=="LABEL" or mn2.startswith("s_branch") or mn2.startswith("s_cbranch"): break
        if mn2=="s_nop": ws+=int(s2.split()[1],0)+1; continue
        srcs=vr2[1:] if vr2 else []
        if "readlane" in mn2 or "readfirstlane" in mn2: srcs=vr2
        if any(not(b[1]<d[0] or b[0]>d[1]) for b in srcs):
            kind=("mfma" if "mfma" in mn2 else "readlane" if "lane" in mn2 else "dpp" if "dpp" in mn2 else "trans" if re.search("rcp|rsq|sqrt|exp|log",mn2) else "ds/mem" if mn2.startswith(("ds_","global_","buffer_","flat_","scratch_")) else "valu")
            if not asm2:
                hits[(kind,ws)]+=1; ex.setdefault((kind,ws),(i+1,s,i2+1,s2))
        if mn2.startswith("v_"): ws+=1
        elif mn2.startswith("s_") and not mn2.startswith("s_waitcnt"): ws+=1
for k,v in sorted(hits.items()): print(k,v,ex[k])
