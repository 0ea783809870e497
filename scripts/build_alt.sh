# Builds libpetdiff.so from git revision REV into scripts/micro/alt/NAME.so (A/B timing against the
# working tree: ALT=NAME.so bash scripts/ab_bench.sh TAG).  Usage: bash scripts/build_alt.sh REV NAME
set -e
REV=${1:?rev}; NAME=${2:?name}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$(mktemp -d /tmp/alt_src.XXXXXX)
git -C "$ROOT" archive "$REV" pet_posterior_distribution_amd/csrc include | tar -x -C "$SRC"
mkdir -p "$ROOT/scripts/micro/alt"
make -C "$SRC/pet_posterior_distribution_amd/csrc" -j8 OUT="$ROOT/scripts/micro/alt/$NAME.so" OBJDIR="$SRC/obj" > "$SRC/build.log" 2>&1 \
  || { tail -20 "$SRC/build.log"; exit 1; }
rm -rf "$SRC"
echo "built scripts/micro/alt/$NAME.so from $REV"
