"""Prints the Zstd decoder's verdict and failure site for every fixture frame
(tests/golden/zstd_*), at capacities 4096 and 49152, through the debug
entry (zstd_uncompress(detail=True)). A GPU-box debugging aid, not a test.
"""
import json, sys, numpy as np, torch
from pathlib import Path
sys.path.insert(0, "/root/repo")
import __graft_entry__ as ge
lvkv = ge.load_package()
g=Path("/root/repo/tests/golden"); spec=json.loads((g/"zstd.json").read_text())
fb=(g/"zstd_frames.bin").read_bytes()
fo=np.concatenate([[0],np.cumsum(spec["frames"])])
dev=torch.device("cuda:0")
for cap in (4096, 49152):
    ks=list(range(len(spec["frames"])))
    fr=[fb[fo[k]:fo[k+1]] for k in ks]
    off=np.concatenate([[0],np.cumsum([len(f) for f in fr])[:-1]]).astype(np.int64)
    src=torch.from_numpy(np.frombuffer(b"".join(fr),dtype=np.uint8).copy()).to(dev)
    d,o,l,st,why=lvkv.zstd_uncompress(src, torch.from_numpy(off).to(dev), torch.tensor([len(f) for f in fr],dtype=torch.int32,device=dev), max_ulen=cap, detail=True)
    torch.cuda.synchronize()
    st=st.cpu().tolist(); why=why.cpu().tolist()
    print(cap, [(k,st[k],why[k]) for k in ks if st[k]!=0][:30])
