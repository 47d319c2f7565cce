"""Per-launch timing of the fine-tune step's grouped GEMMs (csrc/tgemm.hip)
against torch's (rocBLAS) products of the same shapes.

Runs one eager explicit fine-tune step of the bench_train workload, records
every e3gnn_gemm_grouped launch (its problem descriptors), then replays each
recorded launch alone (HIP events over 20 back-to-back calls, median of 5) and the same problems as
torch.addmm calls.  GPU only.

usage: python tools/tgemm_bench.py [--reps 20]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--full', action='store_true', help='print every problem of a long launch')
    a = ap.parse_args()
    from sevennet_finetuning_amd import _lib, train, train_explicit
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    import bench_train
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    model = SevenNetTrainable(device=dev)
    fisher = {n: torch.full_like(p, 1e-3) for n, p in model.named_parameters()}
    opt = {n: p.detach().clone() for n, p in model.named_parameters()}
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': False, 'explicit_grad': True,
           'continue': {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e5}}
    tr = train.Trainer(model, cfg)
    batches = bench_train.make_batches(0, 2, 8, model.chemical_symbols)
    b = [train.collate(x, device=dev, dtype=torch.float32) for x in batches]
    model.train(True)
    tr.rehearsal_step(b[0], b[1])      # warm: workspaces
    rec = []
    orig = train_explicit._Gemms.flush

    def flush(self):
        if self.q:
            rec.append(list(self.q))   # (desc, keep-alive, device, plain operands or None)
        return orig(self)
    train_explicit._Gemms.flush = flush
    tr.rehearsal_step(b[0], b[1])
    train_explicit._Gemms.flush = orig
    torch.cuda.synchronize()
    lib = _lib.load()
    ws = torch.empty(1 << 26, device=dev)

    def timed(fn):
        """per-call time of reps back-to-back calls (the launches queue as in
        the step's graph), median of 5 such runs"""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(10)]
        fn()
        torch.cuda.synchronize()
        for r in range(5):
            ev[2 * r].record()
            for _ in range(a.reps):
                fn()
            ev[2 * r + 1].record()
        torch.cuda.synchronize()
        ts = sorted(ev[2 * r].elapsed_time(ev[2 * r + 1]) * 1e3 / a.reps for r in range(5))
        return ts[2]

    tot_h = tot_t = 0.0
    print(f"{'launch':>6} {'problems (M x N x K[+K2], tA tB; L: irreps layout)':60s} {'tgemm us':>9} {'torch us':>9}")
    for i, q in enumerate(rec):
        n = len(q)
        descs = (_lib.GemmDesc * n)(*[e[0] for e in q])
        shapes = [f"{d.m}x{d.n}x{d.k}{'+' + str(d.k2) if d.k2 else ''}"
                  f"{'L' if d.layout else ('T' if d.trans_a else 'N') + ('T' if d.trans_b else 'N')}"
                  for d in descs]
        stream = torch.cuda.current_stream(dev).cuda_stream
        th = timed(lambda: _lib.check(lib.e3gnn_gemm_grouped(n, descs, ws.data_ptr(), ws.numel(),
                                                             stream)))
        plain = [e[3] for e in q if e[3] is not None]

        def tor():
            for (C, A, B, A2, B2, alpha, beta) in plain:
                torch.addmm(C, A, B, beta=1 if beta else 0, alpha=alpha, out=C)
                if A2 is not None:
                    C.addmm_(A2, B2, alpha=alpha)
        tt = timed(tor) if len(plain) == n else float('nan')
        tot_h += th
        tot_t += tt if tt == tt else 0.0
        print(f"{i:6d} {' '.join(shapes)[:60]:60s} {th:9.1f} {tt:9.1f}")
        if a.full and len(' '.join(shapes)) > 60:
            print(f"{'':6s}   {' '.join(shapes)}")
    print(f"total (one rehearsal step's launches): tgemm {tot_h:.0f} us, torch {tot_t:.0f} us, "
          f"{len(rec)} launches")


if __name__ == '__main__':
    main()
