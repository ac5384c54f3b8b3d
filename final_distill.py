"""Drop-in for the reference's final_distill.py (same flags); see dphubert_amd/cli.py."""
from dphubert_amd.cli import final_distill_main

if __name__ == "__main__":
    final_distill_main()
