"""First on-GPU parity probe: plane batch vs oracle on a few synthetic frames (tools, not product)."""
import ctypes, numpy as np, time, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib.util
spec = importlib.util.find_spec("torch")
ctypes.CDLL(os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so"), mode=ctypes.RTLD_GLOBAL)
P = ctypes.CDLL('pitt_object_table_segmentation_amd/libpitt_seg.so')
O = ctypes.CDLL('oracle/build/libpitt_oracle.so')
import torch
fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
class OP(ctypes.Structure):
    _fields_=[("threshold",ctypes.c_double),("max_iterations",ctypes.c_int32),("probability",ctypes.c_double),("seed",ctypes.c_uint32),("optimize",ctypes.c_int32),("reduce_order",ctypes.c_int32),("trig_mode",ctypes.c_int32),("div_mode",ctypes.c_int32)]
class OR(ctypes.Structure):
    _fields_=[("coefficients",ctypes.c_float*4),("n_coeff",ctypes.c_int32),("hypotheses",ctypes.c_int32),("n_inliers",ctypes.c_int64),("best_hypothesis",ctypes.c_int32),("rejected_samples",ctypes.c_int32),("best_count",ctypes.c_int64),("best_coefficients",ctypes.c_float*4)]
class SP(ctypes.Structure):
    _fields_=[("threshold",ctypes.c_double),("max_iterations",ctypes.c_int32),("probability",ctypes.c_double),("seed",ctypes.c_uint32),("optimize",ctypes.c_int32),("reduce_order",ctypes.c_int32),("div_mode",ctypes.c_int32),("sampler_slack",ctypes.c_int32)]
class PR(ctypes.Structure):
    _fields_=[("coefficients",ctypes.c_float*4),("n_coeff",ctypes.c_int32),("status",ctypes.c_int32),("n_inliers",ctypes.c_int64),("hypotheses",ctypes.c_int32),("best_hypothesis",ctypes.c_int32),("best_count",ctypes.c_int64),("rejected_samples",ctypes.c_int32),("flags",ctypes.c_int32)]
class FR(ctypes.Structure):
    _fields_=[("x",ctypes.c_void_p),("y",ctypes.c_void_p),("z",ctypes.c_void_p),("offsets",ctypes.POINTER(ctypes.c_int64)),("counts",ctypes.POINTER(ctypes.c_int64)),("n_frames",ctypes.c_int32),("capacity",ctypes.c_int64)]
ctx = ctypes.c_void_p()
rc = P.pitt_create(ctypes.byref(ctx), 0); print("create", rc, flush=True)
W,H=640,480; N=W*H
scenes=[(0,1000),(0,1001),(1,1000),(2,1002),(0,1003),(1,1005)]
B=len(scenes)
X=np.empty((B,N),np.float32);Y=X.copy();Z=X.copy()
for i,(sc,sd) in enumerate(scenes): P.pitt_synth_frame(sc, ctypes.c_uint64(sd), W,H, fp(X[i]),fp(Y[i]),fp(Z[i]))
dx=torch.from_numpy(X.reshape(-1)).cuda(); dy=torch.from_numpy(Y.reshape(-1)).cuda(); dz=torch.from_numpy(Z.reshape(-1)).cuda()
inl=torch.empty(B*N,dtype=torch.int32,device='cuda')
offs=(ctypes.c_int64*B)(*[i*N for i in range(B)]); cnts=(ctypes.c_int64*B)(*[N]*B)
fr=FR(dx.data_ptr(),dy.data_ptr(),dz.data_ptr(),offs,cnts,B,B*N)
sp=SP(0.007,1000,0.99,12345,1,0,0,64)
res=(PR*B)()
torch.cuda.synchronize()
t=time.time(); rc=P.pitt_plane_segment_batch(ctx, ctypes.byref(fr), ctypes.byref(sp), res, ctypes.c_void_p(inl.data_ptr())); dt=time.time()-t
P.pitt_last_error.restype=ctypes.c_char_p
print("batch rc", rc, P.pitt_last_error(ctx), "%.3fs"%dt, flush=True)
ginl=inl.cpu().numpy()
ok=True
for i,(sc,sd) in enumerate(scenes):
    op=OP(0.007,1000,0.99,12345,1,0,0,0); r=OR(); oi=np.empty(N,np.int32); hc=np.zeros(1001,np.int32)
    O.orc_plane_segment(fp(X[i]),fp(Y[i]),fp(Z[i]),ctypes.c_int64(N),ctypes.byref(op),oi.ctypes.data_as(ctypes.c_void_p),ctypes.byref(r),hc.ctypes.data_as(ctypes.c_void_p))
    g=res[i]
    gh=np.zeros(1001,np.int32); P.pitt_last_hypothesis_counts(ctx, i, gh.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 1001)
    T=r.hypotheses
    same_counts = np.array_equal(gh[:T], hc[:T])
    gi=ginl[i*N:i*N+g.n_inliers]
    same_inl = g.n_inliers==r.n_inliers and np.array_equal(gi, oi[:r.n_inliers])
    dco = np.max(np.abs(np.array(list(g.coefficients))-np.array(list(r.coefficients))))
    print(f"frame {i} sc{sc}: T gpu {g.hypotheses} cpu {T} best {g.best_hypothesis}/{r.best_hypothesis} cnt {g.best_count}/{r.best_count} "
          f"inl {g.n_inliers}/{r.n_inliers} counts_eq {same_counts} inl_eq {same_inl} dcoef {dco:.3g} status {g.status} flags {g.flags} rej {g.rejected_samples}/{r.rejected_samples}", flush=True)
    if not same_counts:
        bad=np.nonzero(gh[:T]!=hc[:T])[0][:5]; print("  first diffs", bad, gh[bad], hc[bad])
    ok &= same_counts and same_inl and dco==0
print("ALL_OK", ok)
# timing: bigger batch
B2=256
X2=np.tile(X[[0,1,4]].reshape(-1),100)[:B2*N]; 
dx=torch.from_numpy(np.ascontiguousarray(X[[0,1,4]][np.arange(B2)%3].reshape(-1))).cuda()
dy=torch.from_numpy(np.ascontiguousarray(Y[[0,1,4]][np.arange(B2)%3].reshape(-1))).cuda()
dz=torch.from_numpy(np.ascontiguousarray(Z[[0,1,4]][np.arange(B2)%3].reshape(-1))).cuda()
offs=(ctypes.c_int64*B2)(*[i*N for i in range(B2)]); cnts=(ctypes.c_int64*B2)(*[N]*B2)
fr=FR(dx.data_ptr(),dy.data_ptr(),dz.data_ptr(),offs,cnts,B2,B2*N)
res=(PR*B2)()
inl=torch.empty(B2*N,dtype=torch.int32,device='cuda')
for it in range(3):
    P.pitt_plane_segment_batch(ctx, ctypes.byref(fr), ctypes.byref(sp), res, ctypes.c_void_p(inl.data_ptr()))
P.pitt_profile_enable(ctx,1)
t=time.time()
for it in range(10):
    rc=P.pitt_plane_segment_batch(ctx, ctypes.byref(fr), ctypes.byref(sp), res, ctypes.c_void_p(inl.data_ptr()))
dt=time.time()-t
print("256-frame batch: %.3f ms/batch, %.0f frames/s"%(dt/10*1e3, B2*10/dt), "rc", rc)
for k in ["k_hypothesize","k_score","k_replay","k_tile_offsets","k_select_xyz","k_cov_eigen","k_count_final","k_write_final"]:
    l=ctypes.c_int64(); ms=ctypes.c_double(); by=ctypes.c_double()
    P.pitt_profile_get(ctx, k.encode(), ctypes.byref(l), ctypes.byref(ms), ctypes.byref(by))
    print(f"  {k:16s} launches {l.value:5d} total {ms.value:9.3f} ms avg {ms.value/max(1,l.value)*1e3:9.1f} us  GB/s {by.value/max(1e-9,ms.value)/1e6:8.1f}")
