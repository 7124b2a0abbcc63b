# r04: test-before-atomic for the long-row bid minima (ab/bmintest.so) vs the tree, config #3 and #4
set -o pipefail
ITER=2 LIBS="lib ab/bmintest.so" C4=1 bash tools/ab_libs.sh
