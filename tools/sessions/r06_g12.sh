# Round 6 (GPU box): device footprint -- the CLI end to end at first-pass chunk caps
# (r06_g5.sh), then the engine's chunk sweep and k_coop's phase counters (r06_g11.sh)
set -o pipefail
bash tools/sessions/r06_g5.sh && bash tools/sessions/r06_g11.sh
