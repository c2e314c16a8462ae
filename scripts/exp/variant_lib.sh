#!/bin/bash
# Variant library for A/B runs: recompile one source with extra defines and link it with the
# in-tree objects.  scripts/exp/variant_lib.sh <out.so> <source[,source...]> -DNAME=VALUE ...
# Load it with OMF_CODEC_LIB_EXPERIMENT=<out.so> (omnifed_amd/_lib.py).
set -e
cd "$(dirname "$0")/../.."
out=$1; src=$2; shift 2
python3 -m omnifed_amd.build > /dev/null
flags=$(python3 -c "from omnifed_amd.build import FLAGS; print(' '.join(FLAGS))")
objs=()
for o in omnifed_amd/_obj/*.o; do
  b=$(basename $o .o)
  if [[ ",$src," == *",$b,"* ]]; then
    /opt/rocm/bin/hipcc $flags -I include "$@" -c omnifed_amd/csrc/$b -o /tmp/variant_$b.o
    objs+=(/tmp/variant_$b.o)
  else
    objs+=($o)
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" "${objs[@]}"
rm -f "$out".*-amdhsa-* "$out".*-linux-gnu* 2>/dev/null || true
echo "$out"
