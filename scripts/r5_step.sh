set -o pipefail
VARS="main base" REPS=3 B=4096 bash scripts/r5_ab.sh && CLKV="diag_clk:enc" bash scripts/variants/clk_ab.sh
