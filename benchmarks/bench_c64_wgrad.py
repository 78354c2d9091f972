"""64 -> 64 3x3 / stride-1 weight gradient at ResNet-50 layer-1 shape (bs 256, 56 x 56):
own kernel (csrc/hip/conv3x3_c64.hip, bf16 or fp32 twin, incl. its reduce passes) vs MIOpen's
weight-only convolution backward.  One JSON line per dtype."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from vodascheduler_amd.ops import _native as N  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    torch.backends.cudnn.benchmark = True
    h = N.hip()
    n, hh, ww = 256, 56, 56
    cl = torch.channels_last
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(n, 64, hh, ww, device="cuda").to(dt).to(memory_format=cl)
        dy = torch.randn(n, 64, hh, ww, device="cuda").to(dt).to(memory_format=cl)
        w = torch.randn(64, 64, 3, 3, device="cuda").to(dt).to(memory_format=cl)
        dw = torch.zeros(64, 64, 3, 3, device="cuda").contiguous(memory_format=cl)
        ws = torch.empty(h.conv3x3_c64_wgrad_workspace_floats(n, hh), dtype=torch.float32, device="cuda")

        def own():
            h.conv3x3_c64_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *dw.stride(), ws.data_ptr(), n, hh, ww,
                                False, N.dtype_code(dw.dtype), N.stream_of(x), N.dtype_code(x.dtype))

        def lib():
            torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                [False, True, False])

        t_own, t_lib = timeit(own), timeit(lib)
        gflop = 2 * n * hh * ww * 64 * 64 * 9 / 1e9
        ref = torch.nn.grad.conv2d_weight(x[:8].double(), (64, 64, 3, 3), dy[:8].double(), stride=1, padding=1)
        h.conv3x3_c64_wgrad(x[:8].data_ptr(), dy[:8].data_ptr(), dw.data_ptr(), *dw.stride(), ws.data_ptr(), 8, hh,
                            ww, False, N.dtype_code(dw.dtype), N.stream_of(x), N.dtype_code(x.dtype))
        torch.cuda.synchronize()
        rel = float((dw.double() - ref).norm() / ref.norm())
        print(json.dumps({"dtype": str(dt).split(".")[-1], "own_us": round(t_own, 1), "miopen_us": round(t_lib, 1),
                          "own_tf": round(gflop / t_own * 1e3 / 1e3, 1), "miopen_tf": round(gflop / t_lib * 1e3 / 1e3, 1),
                          "rel_err_vs_fp64": rel}), flush=True)


if __name__ == "__main__":
    main()
