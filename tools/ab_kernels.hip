// ab_kernels.hip -- the split-kernel shapes of the round-1..3 study that the
// product library does not dispatch, built only into the A/B library
// (`make -C congestion-control-with-bittorren_amd ab` ->
// build-ab/libsha1chunk.so + libsha1chunk_hip.so, selected with
// SHA1CHUNK_LIB; forced with SHA1CHUNK_SPLIT_UNIT).  Not part of the product:
// these strong definitions replace the product's weak launch_split_study /
// split_unit_study_built (csrc/sha1_kernels.hip), and the shapes come from
// the same templates as the product's (csrc/sha1_split.hpp).  Results:
// profiles/sweep_r01.json, split_variants_r01.json, split_2prod_sweep_r01.json,
// split_unit_ab_r03.json.  Variants that needed code paths of their own and
// lost were removed in round 4 (see the comment at the shape flags).
#include "../congestion-control-with-bittorren_amd/csrc/sha1_split.hpp"

namespace {
constexpr int kStudyUnits[] = {2, 3, 20, 21, 24, 30, 31, 34, 44, 45, 504, 505, 569, 577, 585,
                               8, 9, 10, 12, 13, 16, 17, 86, 87, 91, 92, 93, 94, 95, 96, 97, 98, 99, 81, 82, 83, 84};
}

bool split_unit_study_built(int u) {
    for (int b : kStudyUnits)
        if (u == b) return true;
    return false;
}

hipError_t launch_split_study(const BatchArgs& A, int unit, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t groups = (A.n + 63u) / 64u;
    switch (unit) {
    case 2: hipLaunchKernelGGL((sha1_split_kernel<2, 1>), dim3(groups), dim3(128), 0, st, A); break;
    case 3: hipLaunchKernelGGL((sha1_split_kernel<3, 1>), dim3(groups), dim3(128), 0, st, A); break;
#define SPLIT_V(U, V)                                                                             \
    case 10 * U + V:                                                                              \
        hipLaunchKernelGGL((sha1_split_kernel<U, 1, V>), dim3(groups), dim3(128), 0, st, A);   \
        break;
    // unit 10*U + V, V = kVWK | kVUnmask bits, one producer
    SPLIT_V(2, 0) SPLIT_V(2, 1) SPLIT_V(2, 4) SPLIT_V(3, 0) SPLIT_V(3, 1) SPLIT_V(3, 4)
    SPLIT_V(4, 4) SPLIT_V(4, 5)
#undef SPLIT_V
    // two producer waves per consumer, 4-block units: unit 500 + V
    case 504: hipLaunchKernelGGL((sha1_split_kernel<4, 1, 4, 2>), dim3(groups), dim3(192), 0, st, A); break;
    case 505: hipLaunchKernelGGL((sha1_split_kernel<4, 1, 5, 2>), dim3(groups), dim3(192), 0, st, A); break;
    case 569:  // 500 + (kVWK | kVUnmask | kVSkipWave2): producers on waves 1 and 3
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, 69, 2>), dim3(groups), dim3(256), 0, st, A);
        break;
    case 577:  // 569 + kVRead10 (the product's case 4 without shared loads)
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, 77, 2>), dim3(groups), dim3(256), 0, st, A);
        break;
    case 585:  // the product's case 4 with schedule reads in four bursts of 5
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, (77 & ~kVRead10) | kVCoop, 2>), dim3(groups), dim3(256), 0,
                           st, A);
        break;
    // round 5: the product's uniform case 11 (lane-per-chunk producer loads)
    // with the second pair's read bursts shifted (91), with two bursts of 10
    // (92), and both (93)
    case 91:
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVPhase, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 92:
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVRead10, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 93:
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVRead10 | kVPhase, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;
    case 94:  // one burst of 20, the second pair's at round 40
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVRead20 | kVPhase, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;
    case 95:  // 93 with the shared (coop) producer loads of ragged batches
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V | kVRead10 | kVPhase, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 96:  // 94 with the shared producer loads
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V | kVRead20 | kVPhase, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    // probes (consumer barrier-wait and loop cycles over the digests): the
    // product's uniform case 11 (97), 93 (98), the config-2 case 4 (99)
    case 97:
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVProbe, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 98:
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVRead10 | kVPhase | kVProbe, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;
    case 99:
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, kSplitV<4> | kVProbe, kSplitNProd<4>>), dim3(groups),
                           dim3(256), 0, st, A);
        break;
    case 81:  // 10-read bursts at rounds 10/50 (first pair) and 30/70 (second)
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVRead10 | kVPhase2, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;
    case 82:  // 81 with the probe
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVRead10 | kVPhase2 | kVProbe, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;
    case 83:  // two 4-wave one-pair workgroups per CU, roles by SIMD (kVSimdRole)
        hipLaunchKernelGGL((sha1_split_kernel<2, 1, kVWK | kVUnmask | kVSimdRole, 2>), dim3(groups), dim3(256), 0,
                           st, A);
        break;
    case 84:  // 83 with 10-read bursts
        hipLaunchKernelGGL((sha1_split_kernel<2, 1, kVWK | kVUnmask | kVSimdRole | kVRead10, 2>), dim3(groups),
                           dim3(256), 0, st, A);
        break;
    case 13:  // the product's case 11 with lane-per-chunk producer loads on any layout
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V & ~kVCoop, 2>), dim3((groups + 1) / 2), dim3(512), 0,
                           st, A);
        break;
    // one pair per workgroup, 2-block units, two producers (waves 0, 1, 3 as in
    // case 4): the config-2 layout with case 11's unit size
    case 16:
        hipLaunchKernelGGL((sha1_split_kernel<2, 1, kVWK | kVUnmask | kVSkipWave2 | kVRead10 | kVCoop, 2>),
                           dim3(groups), dim3(256), 0, st, A);
        break;
    case 17:  // case 16 with lane-per-chunk producer loads
        hipLaunchKernelGGL((sha1_split_kernel<2, 1, kVWK | kVUnmask | kVSkipWave2 | kVRead10, 2>), dim3(groups),
                           dim3(256), 0, st, A);
        break;
    case 8:  // 4 pairs per workgroup (512 threads), one consumer + producer per SIMD
        hipLaunchKernelGGL((sha1_split_kernel<1, 4>), dim3((groups + 3) / 4), dim3(512), 0, st, A);
        break;
    case 86:  // case 8 with shared producer loads
        hipLaunchKernelGGL((sha1_split_kernel<1, 4, kVWK | kVUnmask | kVCoop>), dim3((groups + 3) / 4), dim3(512),
                           0, st, A);
        break;
    case 87:  // case 86 with K added in the consumer
        hipLaunchKernelGGL((sha1_split_kernel<1, 4, kVUnmask | kVCoop>), dim3((groups + 3) / 4), dim3(512), 0,
                           st, A);
        break;
    case 10:  // 2 pairs x (consumer + 2 producers), 2-block units, 8-wave layout
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kVWK | kVUnmask | kVLayout8, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 12:  // case 10 with schedule reads in bursts of 10
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kVWK | kVUnmask | kVLayout8 | kVRead10, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;
    case 9:  // 2 pairs per workgroup, 2-block units
        hipLaunchKernelGGL((sha1_split_kernel<2, 2>), dim3((groups + 1) / 2), dim3(256), 0, st, A);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
