"""Build experiment variants of the library (-D flags) into loner_amd/_lib/variants/<tag>.so, for
tools/exp_variants.sh (GPU box) to time under rocprofv3 --stats.

    python tools/exp_variants.py ksb256=LNR_KSB=256 sw2=LNR_SCATTER_WAVES_PER_EU=2,...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv):
    from loner_amd import build as B
    for spec in argv:
        tag, _, defs = spec.partition("=")
        out = os.path.join(ROOT, "loner_amd", "_lib", "variants", tag + ".so")
        B.build(defines=tuple(defs.split(",")), out=out)
        print(tag, "->", out)


if __name__ == "__main__":
    main(sys.argv[1:])
