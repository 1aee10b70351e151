"""GPU idle cost of an event record between dependent kernels on one stream: 200 launches of a
short streaming kernel (tvam_axpy_clamp over n floats) plain, with a timing event recorded after
each, and with a timing-free event after each.  usage: python tools/event_gap.py [n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from drtvam_amd import _abi
    lib = _abi.load_library()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    p = torch.rand(n, device="cuda")
    d = torch.rand(n, device="cuda")
    out = torch.empty_like(p)
    st = torch.cuda.current_stream().cuda_stream
    k = 200

    def run(mode):
        evs = []
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0.record()
        for _ in range(k):
            _abi.check(lib.tvam_axpy_clamp(n, p.data_ptr(), 0.5, d.data_ptr(), 0.0, out.data_ptr(), st))
            if mode == "timing":
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                evs.append(e)
            elif mode == "plain_event":
                e = torch.cuda.Event()
                e.record()
                evs.append(e)
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / k * 1e3

    for rep in range(3):
        for mode in ("none", "timing", "plain_event"):
            print(f"{mode:12s} {run(mode):8.2f} us per launch (n = {n})", flush=True)


if __name__ == "__main__":
    main()
