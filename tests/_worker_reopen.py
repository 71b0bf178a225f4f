"""One member of the iface reopen test: open, barrier, close the same name
ROUNDS times in a row (tests/test_ops_engine.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xucg_amd import ops  # noqa: E402


def main():
    name, rounds = sys.argv[1], int(sys.argv[2])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    for _ in range(rounds):
        it = ops.ShmIface(name, world, rank)
        it.barrier()
        it.close()
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
