"""Reference-compatible entry point: ``python training.py -key K -lr LR [--model ...]``.
See speechrecognitionproject_amd/training.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from speechrecognitionproject_amd.training import main   # noqa: E402

if __name__ == '__main__':
    main()
