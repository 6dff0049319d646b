"""bf16x3-split GEMM (csrc/gemm_x3.hip) vs torch fp32 GEMM: accuracy against
an fp64 reference and time, at the actor MLP's shapes."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-maze_amd"))
import torch  # noqa: E402

from marlmaze import _lib  # noqa: E402
from marlmaze.gemm_tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms()
L = _lib.lib()


def x3(A, B, bias=None, relu=False):
    M, K = A.shape
    N = B.shape[0]
    C = torch.empty(M, N, device=A.device)
    ws = torch.empty(L.mm_gemm_x3_bsplit_len(N, K), dtype=torch.int16, device=A.device)
    _lib.check(L.mm_gemm_x3(_lib.ptr(A), _lib.ptr(B), _lib.ptr(bias), _lib.ptr(C), M, N, K, int(relu),
                            _lib.ptr(ws), _lib.stream_ptr()), "mm_gemm_x3")
    return C


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


M = int(sys.argv[1]) if len(sys.argv) > 1 else 419430
out = {}
torch.manual_seed(0)
for (K, N) in ((460, 264), (264, 264), (264, 460)):
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") * 0.05
    bias = torch.randn(N, device="cuda")
    C = x3(A, B, bias, relu=True)
    Ct = torch._addmm_activation(bias, A, B.t())
    rows = torch.arange(0, M, max(1, M // 2000), device="cuda")
    ref = torch.relu(A[rows].double() @ B.double().t() + bias.double())
    scale = (A[rows].double().abs() @ B.double().abs().t()).clamp_min(1e-30)
    e_x3 = ((C[rows].double() - ref).abs() / scale).max().item()
    e_f32 = ((Ct[rows].double() - ref).abs() / scale).max().item()
    fl = 2.0 * M * N * K
    t_x3 = timeit(lambda: x3(A, B, bias, relu=True))
    t_f32 = timeit(lambda: torch._addmm_activation(bias, A, B.t()))
    r = dict(err_x3=e_x3, err_f32=e_f32, ms_x3=t_x3, ms_f32=t_f32, tf_x3=fl / t_x3 / 1e9, tf_f32=fl / t_f32 / 1e9)
    out[f"M{M} K{K} N{N}"] = r
    print(K, N, json.dumps(r), flush=True)
print(json.dumps(out))
