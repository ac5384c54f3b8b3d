"""Drop-in for the reference's save_final_ckpt.py (same flags); see dphubert_amd/cli.py."""
from dphubert_amd.cli import save_final_ckpt_main

if __name__ == "__main__":
    save_final_ckpt_main()
