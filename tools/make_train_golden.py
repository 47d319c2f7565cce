"""Golden vectors for the fine-tune step, taken from the reference's own
fine-tuning example (read as text; nothing is executed or copied as source):

  example_inputs/fine_tuning/FT_w_reEWC/log.sevenn   "Epoch N/610  lr: X" lines
      -> the cosineannealingwarmuplr schedule (scheduler_param of the same log,
         :67) stepped once per epoch after a fresh reset (reset_scheduler: True)

usage: python tools/make_train_golden.py [/root/reference]
writes tests/golden/ft_lr_schedule.json
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(ref='/root/reference'):
    log = open(os.path.join(ref, 'example_inputs/fine_tuning/FT_w_reEWC/log.sevenn')).read()
    sched = re.search(r"scheduler_param\s*:\s*(\{.*?\})", log).group(1)
    param = json.loads(sched.replace("'", '"'))
    lrs = [(int(e), float(lr))
           for e, lr in re.findall(r'Epoch (\d+)/\d+\s+lr: ([0-9.eE+-]+)', log)]
    out = {'source': 'example_inputs/fine_tuning/FT_w_reEWC/log.sevenn',
           'optim_param': {'lr': 0.0}, 'scheduler': 'cosineannealingwarmuplr',
           'scheduler_param': param, 'printed_decimals': 6,
           'epochs': [e for e, _ in lrs], 'lr': [v for _, v in lrs]}
    path = os.path.join(ROOT, 'tests', 'golden', 'ft_lr_schedule.json')
    with open(path, 'w') as f:
        json.dump(out, f, indent=1)
    print(path, out)


if __name__ == '__main__':
    main(*sys.argv[1:])
