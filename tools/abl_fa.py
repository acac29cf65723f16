import sys, time, os, ctypes
sys.path.insert(0, "/root/repo")
import torch
from paddlepaddle_amd.ops import attention as A, _loader as L
B,S,H,D = 2,2048,40,128
qkv = torch.randn(B,S,H,3,D, device="cuda", dtype=torch.bfloat16)
q,k,v = qkv[:,:,:,0], qkv[:,:,:,1], qkv[:,:,:,2]
o, lse = A._fa_fwd(q,k,v,True,D**-0.5)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
def run(flag):
    dq_acc = torch.empty(B,S,H,D, dtype=torch.float32, device="cuda"); delta = torch.empty(B,H,S, dtype=torch.float32, device="cuda")
    st = A._i64arr(A._strides(q)+A._strides(k)+A._strides(v)+A._strides(o)+A._strides(do)+A._strides(dqkv[:,:,:,0])+A._strides(dqkv[:,:,:,1])+A._strides(dqkv[:,:,:,2]))
    L.call("pa_flash_attn_bwd", L.ptr(q),L.ptr(k),L.ptr(v),L.ptr(o),L.ptr(do),L.ptr(lse),L.ptr(dqkv[:,:,:,0]),L.ptr(dqkv[:,:,:,1]),L.ptr(dqkv[:,:,:,2]),L.ptr(dq_acc),L.ptr(delta),st,B,S,S,H,H,D,D**-0.5,flag,L.stream_ptr())
for flag in (1, -1, 1, -1):
    for _ in range(3): run(flag)
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(20): run(flag)
    torch.cuda.synchronize(); dt=(time.perf_counter()-t)/20
    print("flag", flag, f"{dt*1e3:.3f} ms", f"{2.5*4*B*H*S*S*D/2/dt/1e12:.0f} TF")
