# r04: A/B of the working tree (seq plan loop + per-pass window bid minima +
# summary bitmap) vs the same without the seq loop vs HEAD's build, config #3 and #4
set -o pipefail
ITER=2 LIBS="lib ab/noseq.so ab/base.so" C4=1 bash tools/ab_libs.sh
