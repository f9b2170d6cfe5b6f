import os, sys
sys.path[:0]=['tests','oracle','c-ofdm_amd/python']
import numpy as np, oracle as O, torch
import ofdm_mi355x as M
from common import D
g=O.geometry(D)
nfr=120; pay=g["bytes_per_frame"]-8
body=bytes((i*131+7+(i//pay)*17)&0xFF for i in range(nfr*pay))
frames=[]
for f in range(nfr):
    hdr=np.array([1,0,0,0, f&0xff, f>>8, 0,0],np.uint8)
    data=np.concatenate([hdr,np.frombuffer(body[f*pay:(f+1)*pay],np.uint8)])
    frames.append(O.get_int16(O.frame_write(D,data),D["mult"]).reshape(-1,2))
rng=np.random.default_rng(4); parts=[]
for f in frames:
    parts += [np.zeros((int(rng.integers(0,3001)),2),np.int16), f]
parts.append(np.zeros((g["frame_len"],2),np.int16))
w=np.concatenate(parts).astype(np.float64); x=w[:,0]+1j*w[:,1]
want=O.stream_walk_ring(D,x)[0]
m=M.Modem(D,0)
dx=torch.from_numpy(x).cuda()
for tun in (dict(), dict(exact_search=1), dict(t2_f32=0), dict(t2_f32=0, exact_search=1)):
    m.walk_tuning(**tun)
    for chunk in (0, 2000000):
        pb=torch.full((200,),-1,dtype=torch.int64,device="cuda")
        nf=m.rx_stream(dx,len(x),200,pb_out=pb,chunk=chunk)
        torch.cuda.synchronize()
        got=pb[:nf].cpu().numpy()
        print(tun,"chunk",chunk,"nf",nf,"want",len(want),"equal",np.array_equal(got,want), flush=True)
        if not np.array_equal(got,want):
            print(" missing", sorted(set(want)-set(got))[:20], " extra", sorted(set(got)-set(want))[:20], flush=True)
# the first missing frame: oracle detail
pb0 = sorted(set(want))[0]
print("x amplitude", np.abs(x).max())
