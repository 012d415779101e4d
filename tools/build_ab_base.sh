# A/B helper: ab/libkdfm_base.so = the current objects with the listed csrc files taken from a git revision
# usage: bash tools/build_ab_base.sh REV file.hip [file.hip ...]   (run after building the current library)
set -e
REV=$1; shift
D=/tmp/kdfm_ab_base
rm -rf $D && mkdir -p $D/obj
cp kd-via-fm-in-asr_amd/csrc/build/*.o $D/obj/
for f in "$@"; do
  git show $REV:kd-via-fm-in-asr_amd/csrc/$f > kd-via-fm-in-asr_amd/csrc/.ab_$f
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -munsafe-fp-atomics -Wno-unused-result \
    -Iinclude -c kd-via-fm-in-asr_amd/csrc/.ab_$f -o $D/obj/${f%.hip}.o
  rm -f kd-via-fm-in-asr_amd/csrc/.ab_$f
done
mkdir -p ab
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ab/libkdfm_base.so $D/obj/*.o -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx
echo "ab/libkdfm_base.so: $REV $*"
