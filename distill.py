"""Drop-in for the reference's distill.py (same flags); see dphubert_amd/cli.py."""
from dphubert_amd.cli import distill_main

if __name__ == "__main__":
    distill_main()
