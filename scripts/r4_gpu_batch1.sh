#!/bin/bash
# mask A/B (affects the default backward), then the forward PMC passes
set -o pipefail
bash scripts/r4_hs_mask_ab.sh || exit 1
SHAPE="96 25 512 64 1" TAG=xl bash scripts/fa_fwd_pmc.sh && SHAPE="4 16 4096 64 1" TAG=n4096c bash scripts/fa_fwd_pmc.sh && SHAPE="4 16 4096 64 0" TAG=n4096 bash scripts/fa_fwd_pmc.sh
