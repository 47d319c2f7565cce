"""CPU oracle for the SevenNet-0 energy/force hot path -- TEST INFRASTRUCTURE ONLY.

This package is the *checker*, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The shipped path (``sevennet_finetuning_amd``) never imports,
links or executes anything under ``oracle/`` and fails loudly when its HIP
library is missing.

Contents
--------
* ``cg``            -- real-basis Clebsch-Gordan tables in e3nn's convention
                       (Racah formula + real/complex change of basis), with the
                       per-triple sign convention pinned to the frozen tables of
                       the reference deployment (tests/golden/cg_frozen.npz).
* ``sevennet_ref``  -- plain-PyTorch (fp32 or fp64, CPU) restatement of
                       SevenNet-0's forward pass and autograd force/stress, each
                       function citing the reference file:line it follows.
* ``neighbor``      -- O(N^2)/cell-list periodic neighbor list with the
                       reference's edge convention (dataload.py:113-125).

Parity pinning
--------------
The reference's Python package cannot be imported here (e3nn/ase/PyG absent,
ModuleNotFoundError) and its frozen TorchScript deployments are *not* executed
by this build (they are serialized programs; we only read them as text/raw
bytes).  The restatement is pinned by the known-answer values the survey
measured with the reference's own frozen model, kept in
``tests/golden/kat_reference.json``, and by the frozen CG tables (raw float32
bytes of the deployment's constant storages, ``tests/golden/cg_frozen.npz``).
"""
