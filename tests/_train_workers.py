"""Spawned ranks for the multi-rank fine-tune GPU test (test_gpu_train.py):
two gloo ranks on the box's GPU running the DDP rehearsal step eagerly or as
captured HIP-graph segments around the gradient all-reduces."""
import os

import numpy as np
import torch


def ddp_rehearsal_worker(rank, world, port, graph, out):
    import torch.distributed as dist
    from sevennet_finetuning_amd import train
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    from test_gpu_train import DEV, _batch
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    m = SevenNetTrainable(device=DEV)
    fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
    opt = {n: p.detach().clone() for n, p in m.named_parameters()}
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99}, 'device': DEV, 'hip_graph': graph,
           'is_ddp': True,
           'continue': {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e5}}
    tr = train.Trainer(m, cfg)
    m.train(True)

    def coll(seeds):
        return train.collate(_batch(seeds), device=DEV, dtype=torch.float32)
    # equal shapes on every step and rank (one captured signature per rank),
    # different data per rank
    s0 = 20 * rank
    pairs = [(coll([s0 + 1]), coll([s0 + 2])), (coll([s0 + 3]), coll([s0 + 4]))]
    losses = [[float(x) for x in tr.rehearsal_step(*pairs[i % 2])] for i in range(4)]
    n_graphs = len(tr._graphed.cache) if tr._graphed is not None else 0
    np.savez(out + f'.{rank}.npz', losses=np.array(losses),
             flat=m.flat.detach().double().cpu().numpy(), n_graphs=n_graphs)
    dist.barrier()
    dist.destroy_process_group()
