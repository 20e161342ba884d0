"""Entry point with the reference's name and no-arg behaviour (reference ``predict_hf.py``).

    python predict_hf.py                      # prints 27.09 % for the shipped example patient
    python predict_hf.py --set Dyspnea=1 --device cuda
"""
import sys

from hfens.cli.predict_hf import main

if __name__ == "__main__":
    sys.exit(main())
