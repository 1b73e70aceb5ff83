# round-6 A/B batch: the (2,4) tree-block solve for non-arrowhead substeps; (2,8) at 7 arenas per CU
set -o pipefail
bash tools/ab_tb24.sh && bash tools/ab_gl28.sh
