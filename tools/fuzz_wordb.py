#!/usr/bin/env python3
"""Fuzz of the drop-in adapter's rule for word-boundary tables
(integration/reflex_gpu_matcher.h predictor_exact): random patterns with
\\b \\B \\< \\> around finite and looping bodies; for every pattern the rule
sends to the GPU (finite language, no boundary-dependent accept that goes on
with bytes: ugpu_dfa_info.shape), the reference as ugrep runs it
(oracle/_ref/ref_harness mode "re") must equal the reference with its match
predictor off (mode "reP": the DFA semantics the engine implements) on the
inputs below.  Build container only (needs the reference harness).

    python tools/fuzz_wordb.py SEED COUNT    -> "ok N bad 0 skip M"
"""
import random, subprocess, json, sys
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
import numpy as np
import ugrep_amd as U
from ugrep_amd.matcher import host_context
H='/root/repo/oracle/_ref/ref_harness'
rnd=random.Random(int(sys.argv[1]) if len(sys.argv)>1 else 1)
B=['\\b','\\B','\\<','\\>','']
atoms=['a','b','ab','foo','_','1','é','x','[a-z]','\\w','\\d','.','[^a ]','(a|bc)','(fo|foo)','\\s','[0-9_]',"it's"]
def body():
    k=rnd.randint(1,3); s=''
    for _ in range(k):
        a=rnd.choice(atoms)
        r=rnd.random()
        if r<0.15: a='(?:%s){1,2}'%a
        elif r<0.25: a=a+'?'
        elif r<0.35: a=a+'+'
        elif r<0.4: a=a+'*'
        s+=a
    return s
def pat():
    s=rnd.choice(B)+body()+rnd.choice(B)
    if rnd.random()<0.25: s+='|'+rnd.choice(B)+body()+rnd.choice(B)
    return s
def props(opc):
    try:
        tab=U.host_tables(opc)
    except U.Unsupported:
        return None
    info=tab['info']
    acap,anch,_=host_context(opc)
    nctx=info['contexts']; S=info['states']; row=info['row']
    trans=tab['trans']; cls=tab['cls']
    # successors
    succ=[set() for _ in range(S)]
    for s in range(S):
        for c in range(256):
            col=c if info['format']==0 else int(cls[c])
            t=int(trans[s*row+col])//row
            if t: succ[s].add(t)
    # cycle detection (reachable from start)
    start=tab['start']//row
    color=[0]*S; cyc=False
    sys.setrecursionlimit(100000)
    def dfs(u):
        nonlocal cyc
        color[u]=1
        for v in succ[u]:
            if color[v]==1: cyc=True
            elif color[v]==0: dfs(v)
        color[u]=2
    dfs(start)
    condedge=False
    if nctx==64:
        for s in range(S):
            row_=acap[s*64:(s+1)*64]
            if len(set(int(x) for x in row_))>1 and succ[s]: condedge=True
    return dict(cyc=cyc, condedge=condedge, nctx=nctx)
inputs=['gen:3:1:0:100000','gen:4:1:0:100000','file:/root/repo/tests/golden/lorem.utf8.txt']
ok=bad=skip=0
for i in range(int(sys.argv[2]) if len(sys.argv)>2 else 200):
    p=pat()
    d=subprocess.run([H,'dump','re',p],capture_output=True,text=True)
    if d.returncode: skip+=1; continue
    opc=json.loads(d.stdout)['opc']
    pr=props(opc)
    if pr is None or pr['nctx']!=64: skip+=1; continue
    eligible = not pr['cyc'] and not pr['condedge']
    diff=False
    for inp in inputs:
        a=subprocess.run([H,'find','re',p,inp],capture_output=True,text=True).stdout
        b=subprocess.run([H,'find','reP',p,inp],capture_output=True,text=True).stdout
        if a!=b: diff=True; break
    if eligible and diff: bad+=1; print('ELIGIBLE BUT DIFF', repr(p))
    elif eligible: ok+=1
    else: skip+=1
print('ok',ok,'bad',bad,'skip',skip)
