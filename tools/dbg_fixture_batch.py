import sys, numpy as np
sys.path.insert(0,"tests"); sys.path.insert(0,"parquet-mr_amd"); sys.path.insert(0,".")
from fixtures import chunk_cases, load_chunk
from pqgpu import abi, decoder as D
from tools.synth import writer
CASES=list(chunk_cases())
chunks=[];exps=[];names=[]
for name,c in CASES:
    ch,e=load_chunk(name,c)
    if ch.physical_type==abi.BYTE_ARRAY: continue
    chunks.append(ch); exps.append(np.asarray(e)); names.append((name,c['key'],c['path']))
dec=D.Decoder(0)
def run(idx):
    b=writer.build_batch([chunks[i] for i in idx])
    cols,st=dec.decode(dec.upload(b), check=False)
    bad=[]
    for k,i in enumerate(idx):
        g=np.asarray(cols[k].numpy()); e=exps[i]
        if g.dtype.kind=='f': g=g.view(np.uint64 if g.itemsize==8 else np.uint32); e=e.view(g.dtype)
        m=np.nonzero(g!=e)[0]
        if m.size: bad.append((i,names[i],m[:5].tolist(), g[m[:3]].tolist(), e[m[:3]].tolist(), [int(np.nonzero(e==x)[0][:3].tolist()[0]) if (e==x).any() else -1 for x in g[m[:3]]]))
    return st.code, bad
print("all", run(list(range(len(chunks)))))
print("21 alone", run([21]))
for j in range(len(chunks)):
    if j==21: continue
    c,b=run([j,21])
    if b: print("pair",j,names[j],c,b)
for j in range(len(chunks)):
    c,b=run([j])
    if b: print("single",j,c,b)
