# Build porqua_amd/libporqua_hip_old.so from a committed revision (default HEAD) for an A/B
# against the working tree, without touching the working tree: bash tools/build_old_lib.sh [rev]
set -e
REV=${1:-HEAD}
D=$(mktemp -d /tmp/pq_old.XXXX)
git archive "$REV" porqua_amd/csrc include | tar -x -C "$D"
make -C "$D/porqua_amd/csrc" -j8 BUILD=build LIB="$(pwd)/porqua_amd/libporqua_hip_old.so" > "$D/make.log" 2>&1
rm -rf "$D"
echo "built porqua_amd/libporqua_hip_old.so from $(git rev-parse --short "$REV")"
