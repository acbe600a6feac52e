# the failing vector through older trees (git worktrees under bisect/, each with its own libraries)
set -o pipefail
R=$PWD
for c in "$@"; do
  (cd bisect/$c && MI_VDIR=$R/sweep_one GRAFT_REPO_ROOT=$R/bisect/$c timeout -k 10 120 python -u $R/tools/dev/one_vector.py test15549_5522_4902 | sed "s/^/$c /") || { echo "$c failed"; exit 1; }
done
