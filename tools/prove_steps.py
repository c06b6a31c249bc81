"""Per-step prove timings and device memory (diagnostic):
python tools/prove_steps.py [steps] [bench.py options, e.g. --vector-len 1]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    args = bench.make_parser().parse_args(sys.argv[2:])
    from plonky3_eon_amd import Context

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    wl = bench.ProveWorkload(args, ctx, dev, 0)
    for i in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wl.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        free, total = torch.cuda.mem_get_info()
        print(f"step {i}: {dt:.1f} ms  free {free / 2**30:.1f} GiB of {total / 2**30:.1f}  "
              f"torch alloc {torch.cuda.memory_allocated() / 2**30:.1f} reserved {torch.cuda.memory_reserved() / 2**30:.1f}  "
              f"{ {k: round(v, 1) for k, v in wl.timings[-1].items()} }", flush=True)


if __name__ == "__main__":
    main()
