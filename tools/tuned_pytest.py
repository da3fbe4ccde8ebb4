"""Run pytest in-process with library tunings set first (A/B correctness of
a tuning-gated kernel variant before it becomes a default):
    python tools/tuned_pytest.py KEY=VAL[,KEY=VAL] <pytest args...>
Test infrastructure only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vaeunet_amd import _lib
    for kv in filter(None, sys.argv[1].split(",")):
        k, v = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(k), int(v))
    import pytest
    sys.exit(pytest.main(sys.argv[2:]))


if __name__ == "__main__":
    main()
