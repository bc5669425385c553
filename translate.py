#!/usr/bin/env python
"""Drop-in for the reference's translate.py CLI (achilles1989/NanoDecoder
translate.py:173-187) running the MI355X engine, e.g.

    python translate.py -model model.pt -src_dir reads/ -save_data out/ -gpu 0 \\
        -src_seq_length 512 -fast -beam_size 5 -batch_size 100
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from nanodecoder_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    import warnings

    warnings.simplefilter("ignore")
    main()
