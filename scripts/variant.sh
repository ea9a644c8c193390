#!/bin/bash
# Build an A/B variant of the engine: build/var/<name>/libsda_engine.so, reusing the default
# objects except those listed (rebuilt with EXTRA flags).   Run it with SDA_ENGINE_LIB=<that .so>.
#   bash scripts/variant.sh <name> "<extra hipcc flags>" packed_gen_27 [more objects]
set -e
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=$2; shift 2
D=build/var/$NAME
rm -rf $D; mkdir -p $D/obj
cp build/obj/*.o $D/obj/
for o in "$@"; do rm -f $D/obj/$o.o; done
make -s OBJDIR=$D/obj LIB=$D/libsda_engine.so EXTRA="$EXTRA" $D/libsda_engine.so
echo "built $D/libsda_engine.so"
