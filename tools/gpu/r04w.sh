# gate LDS cap 36 / 40 KB per 4 waves vs 44 (default), two alternations
set -o pipefail
bash tools/gpu/exp.sh r04w/ab1 kb36 kb40 || exit 1
bash tools/gpu/exp.sh r04w/ab2 kb40 kb36 || exit 1
