#!/bin/bash
# CPU side: ablation builds of libxfgstark.so for the configs[4] LDE (ab/lib_<variant>.so, loaded
# on the GPU box with XFG_LIB): the NTT passes with their arithmetic (DFT butterflies, twiddle and
# pre-factor multiplies) or their global stores removed, to split a pass's time into its memory
# skeleton and its arithmetic. Output is wrong by construction: timing only.
set -e
cd "$(dirname "$0")/.."
make -s -C xfg-stark_amd build/kernels.hip.o build/prover.hip.o build/verify_kernels.hip.o build/verifier.cpp.o
for v in nomath nostore; do
  sed -e 's/^\(\s*\)dft_reg<LOGR, INV>(v\[q\]);/\1ABL_M(dft_reg<LOGR, INV>(v[q]));/' \
      -e 's/for (int r = 1; r < R; r++) v\[q\]\[r\] = gl_mul(v\[q\]\[r\], TW2D/for (int r = 1; r < R \&\& ABL_MATH == 0; r++) v[q][r] = gl_mul(v[q][r], TW2D/' \
      -e 's/^\(\s*\)y\[((u64)(base + r \* stride) << rs) + cb\] = gl_mul(v\[r\], w);/\1if (ABL_STORE == 0 || a.keep == 12345) y[((u64)(base + r * stride) << rs) + cb] = ABL_MATH ? v[r] : gl_mul(v[r], w);/' \
      -e 's/^\(\s*\)buf_st(rout, (seq + ((u32)base << a.logR)) \* 8, ((u32)(r \* stride) << a.logR) \* 8, canon(v\[r\]));/\1if (ABL_STORE == 0 || a.keep == 12345) buf_st(rout, (seq + ((u32)base << a.logR)) * 8, ((u32)(r * stride) << a.logR) * 8, ABL_MATH ? v[r] : canon(v[r]));/' \
      -e 's/return gl_mul(v, preg ? preg\[j + o\] : pre\[j + o\]);/return ABL_MATH ? v : gl_mul(v, preg ? preg[j + o] : pre[j + o]);/' \
      xfg-stark_amd/csrc/ntt.hip > ab/ntt_$v.hip
  M=0; S=0; [ $v = nomath ] && M=1; [ $v = nostore ] && S=1
  sed -i "1i #define ABL_MATH $M\n#define ABL_STORE $S\n#define ABL_M(...) do { if (!ABL_MATH) { __VA_ARGS__; } } while (0)" ab/ntt_$v.hip
  grep -c "ABL_" ab/ntt_$v.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I xfg-stark_amd/csrc -c ab/ntt_$v.hip -o ab/ntt_$v.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ab/lib_$v.so xfg-stark_amd/build/kernels.hip.o ab/ntt_$v.o xfg-stark_amd/build/prover.hip.o xfg-stark_amd/build/verify_kernels.hip.o xfg-stark_amd/build/verifier.cpp.o
done
ls -la ab/*.so
