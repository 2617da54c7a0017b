# Build the working tree's library with extra compile flags as a named A/B variant:
#   bash tools/ab_variant.sh <name> "-DSGCN_X=1 ..."  ->  tools/ab/libshiftgcn_hip_<name>.so
# (through the Makefile's `diag` target: its own objects and output name; a variant built
# with a diagnostic macro reports SGCN_ABI_DIAG_FLAG and loads only with
# SGCN_ALLOW_DIAG_LIB=1)
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
rm -rf /tmp/sgcn_var_$1 && mkdir -p /tmp/sgcn_var_$1 $ROOT/tools/ab
cp -r $ROOT/shift-gcn_amd/csrc $ROOT/include /tmp/sgcn_var_$1/
mkdir -p /tmp/sgcn_var_$1/shift-gcn_amd && mv /tmp/sgcn_var_$1/csrc /tmp/sgcn_var_$1/shift-gcn_amd/
rm -rf /tmp/sgcn_var_$1/shift-gcn_amd/csrc/build /tmp/sgcn_var_$1/shift-gcn_amd/csrc/build_diag
make -C /tmp/sgcn_var_$1/shift-gcn_amd/csrc -j8 diag DIAG="$2" \
  DIAG_OUT=$ROOT/tools/ab/libshiftgcn_hip_$1.so > /dev/null
echo built tools/ab/libshiftgcn_hip_$1.so with "$2"
