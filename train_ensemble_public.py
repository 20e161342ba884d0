"""Entry point with the reference's name (reference ``train_ensemble_public.py``).

    python train_ensemble_public.py                         # .mat files next to this script, else synthetic
    python train_ensemble_public.py --device cuda --rows 10000 --features 40 --timings
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train_ensemble_public.py --rows 100000
"""
import os
import sys

from hfens.cli.train_ensemble_public import main

if __name__ == "__main__":
    sys.exit(main(script_dir=os.path.dirname(os.path.abspath(__file__))))
