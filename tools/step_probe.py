import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
import numpy as np, torch, ctypes as C
from scipy.special import expit
from nemo import generator, _lib
from nemo.engine import Engine
from nemo.nem_order_mcmc import SIG0, SIG1
m = generator.config_nem("C3"); eng = Engine.for_nem(m)
for opt in ("graphs", "local_split", "exact", "exact_cform", "exact_xcd", "exact_form", "anc_overlap"):
    if opt.upper() in os.environ:
        eng.set_option(opt, int(os.environ[opt.upper()]))
S = 64; n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
rng = np.random.default_rng(3)
pos = np.array([rng.permutation(S) for _ in range(n)], dtype=np.int32)
w = rng.uniform(-3, 3, (n, S, S)); w01 = expit(w)
anc = np.clip(rng.random((n, S, S)) - 0.5, 0, 1)
eng.optimal_weights(pos, w01, anc, w, SIG0, SIG1, raise_on_fail=False)
def med(f, k=30):
    ts = []
    for _ in range(k):
        t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
    return 1e3 * np.median(ts)
print("wrapper", med(lambda: eng.optimal_weights(pos, w01, anc, w, SIG0, SIG1, raise_on_fail=False)))
lib = _lib.load()
wn = w.copy(); ll1 = np.empty(n); lld = np.empty(n); info = np.empty((n, S, S), dtype=np.int32)
P = lambda a, t=C.c_double: a.ctypes.data_as(C.POINTER(t))
def raw(): lib.nemo_optimal_weights(eng._ctx, n, P(pos, C.c_int32), P(w01), P(anc), SIG0, SIG1, 0, P(wn), P(ll1), P(lld), P(info, C.c_int32))
print("raw ctypes", med(raw))
dp = torch.from_numpy(pos).cuda(); dw = torch.from_numpy(w01).cuda(); da = torch.from_numpy(anc).cuda()
dn = torch.from_numpy(w).cuda(); d1 = torch.zeros(n, dtype=torch.float64, device="cuda"); d2 = torch.zeros_like(d1)
di = torch.zeros((n, S, S), dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
def dev():
    lib.nemo_optimal_weights_dev(eng._ctx, n, C.c_void_p(dp.data_ptr()), C.c_void_p(dw.data_ptr()), C.c_void_p(da.data_ptr()), SIG0, SIG1, 0, C.c_void_p(dn.data_ptr()), C.c_void_p(d1.data_ptr()), C.c_void_p(d2.data_ptr()), C.c_void_p(di.data_ptr()), C.c_void_p(st))
    torch.cuda.synchronize()
print("dev only", med(dev))
def dev10():
    for _ in range(10):
        lib.nemo_optimal_weights_dev(eng._ctx, n, C.c_void_p(dp.data_ptr()), C.c_void_p(dw.data_ptr()), C.c_void_p(da.data_ptr()), SIG0, SIG1, 0, C.c_void_p(dn.data_ptr()), C.c_void_p(d1.data_ptr()), C.c_void_p(d2.data_ptr()), C.c_void_p(di.data_ptr()), C.c_void_p(st))
    torch.cuda.synchronize()
print("dev x10 / 10", med(dev10, 10) / 10)
# A/B of one option on the synchronous staged call, interleaved (AB_OPT=name:
# rounds of 30 calls with the option at 0 and 1 in turn; medians per value)
if os.environ.get("AB_OPT"):
    name = os.environ["AB_OPT"]
    vals = [int(v) for v in os.environ.get("AB_VALS", "0,1").split(",")]
    res = {v: [] for v in vals}
    for _ in range(7):
        for v in vals:
            eng.set_option(name, v)
            raw()  # first call after an option change captures a new graph
            res[v].append(med(raw))
    for v in vals:
        print(f"AB {name}={v} raw ctypes median of rounds {np.median(res[v]):.5f} ms, rounds {np.round(res[v], 5).tolist()}")
    eng.set_option(name, vals[-1])
# the step from W (W~ and ancestor_x made on the device)
print("from W (wrapper)", med(lambda: eng.optimal_weights_w(pos, w, SIG0, SIG1, raise_on_fail=False)))
