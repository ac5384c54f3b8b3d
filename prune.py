"""Drop-in for the reference's prune.py (same flags); see dphubert_amd/cli.py."""
from dphubert_amd.cli import prune_main

if __name__ == "__main__":
    prune_main()
