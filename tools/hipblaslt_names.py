"""Which hipBLASLt kernels torch picks for the UNet's dominant GEMM shapes (run under
rocprofv3 --kernel-trace --stats): the kernel names encode the library's tile / depth / wave
configuration, a yardstick for tuning the ring GEMM."""
import torch

SHAPES = [(8192, 10240, 1280), (8192, 1280, 5120), (8192, 3840, 1280), (32768, 5120, 640), (32768, 640, 2560), (8192, 1280, 1280)]


def main():
    dev = torch.device("cuda")
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        for _ in range(5):
            torch.nn.functional.linear(x, w)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
