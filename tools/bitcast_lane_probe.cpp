// Probe of the ROCm 7.2 clang lowering that caused the round-4 "wrong dy" (tools/isa_hazard_check.py
// --bitcast-lanes): __builtin_bit_cast of an ext_vector_type element lvalue reads element 0.  Two forms:
// the subscript v[2] and the swizzle accessor v.z (the same element through an ext_vector lane name).
//   /opt/rocm/lib/llvm/bin/clang++ -O2 tools/bitcast_lane_probe.cpp -o /tmp/p && /tmp/p
// prints "affected" (exit 1) when either form differs from a bit_cast of a named temporary, "fixed" (exit 0)
// otherwise.
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__attribute__((noinline)) unsigned lane2_bits(f4 v) { return __builtin_bit_cast(unsigned, v[2]); }
__attribute__((noinline)) unsigned lane2_bits_swz(f4 v) { return __builtin_bit_cast(unsigned, v.z); }
__attribute__((noinline)) unsigned lane2_bits_tmp(f4 v) { const float t = v[2]; return __builtin_bit_cast(unsigned, t); }
int main() {
    const f4 v = {1.f, 2.f, 3.f, 4.f};
    const unsigned a = lane2_bits(v), s = lane2_bits_swz(v), b = lane2_bits_tmp(v);
    const bool ok = a == b && s == b;
    printf("bit_cast(v[2]) = 0x%08x, bit_cast(v.z) = 0x%08x, via a temporary 0x%08x: %s\n", a, s, b,
           ok ? "fixed" : "affected");
    return ok ? 0 : 1;
}
