"""Per-kernel PMC digest of tools/pmc_bk.sh output: wait/active fractions,
LDS bank conflicts, instruction counts and HBM-side GB (FETCH_SIZE x 2 per
MI355X_MICROARCH.md; WRITE_SIZE as is), L2 hit rate.

  python tools/pmc_bk_summary.py gpurun_out/pmc_bk7 [kernel-substring ...]
"""
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_summary import load  # noqa: E402


def main():
    root = sys.argv[1]
    subs = sys.argv[2:] or ["k_bk_"]
    per, launches = load(root)
    for name in sorted(per, key=lambda n: -per[n].get("SQ_BUSY_CYCLES", 0)):
        if not any(s in name for s in subs):
            continue
        c = per[name]
        wc = max(1.0, c.get("SQ_WAVE_CYCLES", 0))
        short = name.split("(")[0].replace("void ", "")
        print("%s" % short)
        print("   wait_any %.2f wait_inst %.2f active %.2f wait_lds %.2f lds_bank/active %.2f"
              % (c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc,
                 c.get("SQ_ACTIVE_INST_ANY", 0) / wc, c.get("SQ_WAIT_INST_LDS", 0) / wc,
                 c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0))))
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        print("   valu %.3g salu %.3g lds %.3g vm_rd %.3g vm_wr %.3g | fetch %.1f GB write %.1f GB l2_hit %.2f"
              % (c.get("SQ_INSTS_VALU", 0), c.get("SQ_INSTS_SALU", 0), c.get("SQ_INSTS_LDS", 0),
                 c.get("SQ_INSTS_VMEM_RD", 0), c.get("SQ_INSTS_VMEM_WR", 0),
                 c.get("FETCH_SIZE", 0) * 1024 * 2 / 1e9, c.get("WRITE_SIZE", 0) * 1024 / 1e9,
                 hit / max(1.0, hit + miss)))


if __name__ == "__main__":
    main()
