"""Where did the ranks' collective sequences part? Reads the flight-recorder files that
PADDLE_AMD_COLLECTIVE_TRACE_DIR makes every rank write (distributed/collective_check.py) and prints, per
communicator, the first entry at which two members differ or the members that stopped early (a hang).

    python tools/collective_trace_diff.py <trace dir>
"""
import glob
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddlepaddle_amd.distributed.collective_check import first_divergence  # noqa: E402


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "."
    paths = sorted(glob.glob(os.path.join(d, "collectives.rank*.log")))
    if not paths:
        raise SystemExit(f"no collectives.rank*.log under {d}")
    found = first_divergence(paths)
    print("\n".join(found) if found else f"{len(paths)} ranks: sequences agree")
    sys.exit(1 if found else 0)


if __name__ == "__main__":
    main()
