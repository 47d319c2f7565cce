"""Diagnostic (round 3): a large torch.sum (PyTorch's multi-block "global"
reduction, whose semaphores are zeroed by a hipMemsetAsync before each launch)
captured in a HIP graph, replayed with and without other reductions between
the replays.  Prints the graph's result against an eager recomputation, and
the same for the two-level form the EWC loss now uses (rows of 1024 reduced
per block, then the row sums): the graph must reproduce the eager value on
every replay."""
import torch

dev = torch.device('cuda', 0)
N = 842623
g0 = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(N, device=dev, generator=g0)
y = torch.randn(N, device=dev, generator=g0)


def two_level(v):
    m = v.numel() // 1024 * 1024
    return v[:m].view(-1, 1024).sum(1).sum() + v[m:].sum()


for name, fn in (('torch.sum', lambda v: (v * v).sum()), ('two-level', lambda v: two_level(v * v))):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn(x)
    for mode in ('alone', 'interleaved', 'interleaved+sync'):
        errs = []
        for i in range(6):
            x.mul_(1.01)   # new input each replay
            g.replay()
            got = out.clone()
            if mode != 'alone':
                _ = fn(y)          # another (eager) reduction of the same shape
                if mode.endswith('sync'):
                    torch.cuda.synchronize()
            ref = fn(x)
            errs.append(float((got - ref).abs() / ref.abs()))
        print(f'{name:10s} {mode:17s} max rel err over 6 replays: {max(errs):.3e}  '
              f'{["%.1e" % e for e in errs]}', flush=True)
