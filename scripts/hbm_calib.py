"""Calibrate achievable HBM bandwidth on this GPU with torch's own kernels.

Write-only (fill_) and read+write (copy_) over multi-GB buffers, HIP-event timed.
Prints one JSON line (GB/s) so the kernels' achieved rates can be read against what the
chip sustains, not only against the 8 TB/s spec peak."""
import json

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    n = 8 << 30
    x = torch.empty(n, dtype=torch.uint8, device='cuda')
    fill = n / timed(lambda: x.fill_(1)) / 1e9
    half = n // 2
    src, dst = x[:half], x[half:]
    copy = 2 * half / timed(lambda: dst.copy_(src)) / 1e9
    y = x.view(torch.float64)
    fill64 = n / timed(lambda: y.fill_(1.5)) / 1e9
    print(json.dumps({'fill_u8_GBs': round(fill, 1), 'fill_f64_GBs': round(fill64, 1),
                      'copy_GBs_read_plus_write': round(copy, 1), 'bytes': n}))


if __name__ == '__main__':
    main()
