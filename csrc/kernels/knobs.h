// Runtime tuning / diagnostic knobs of libtcamd_hip.so (one registry).
//
// Every knob a host entry point consults lives in the table in
// csrc/runtime/knobs.hip: name, default and what it steers.  A knob starts at
// its environment variable (read once, at the first lookup) or its default,
// and can be changed at run time through tcamd_knob_set -- the tests switch
// paths in-process that way instead of spawning a process per setting.  A
// value is read at launch time: a HIP graph keeps the kernels (and the
// variants) it captured.  README "Tuning knobs" lists each with its test;
// tests/test_knobs.py keeps the table, the sources and the README in sync.
#pragma once

namespace tcamd {

enum class Knob : int {
  X3Bm = 0,        // K8x 1x1 tile rows (32 / 64 / 128; 0 = by size)
  X3SplitkBelow,   // K8x split-K when fewer tiles than this
  X3MaxSplits,     // K8x split-K cap
  X3Ws,            // K8x warp-specialised persistent 1x1 (0 = tiled kernel only)
  X3WsMin,         // ... from this many pixels
  X3StemBpc,       // K10x stem persistent blocks per CU
  X3sBlocks,       // K13x 1x1 target workgroups
  X3sMaxChunks,    // K13x 1x1 K-chunk cap
  X3sSplit3,       // K13x 3x3 over input quarters (0 = one block, bitwise reproducible)
  PkBigLim,        // K2 pack: output offset past which a block takes the 64-bit byte path
  K3Mode,          // K3 index: 1 = general walk only
  K17Tm,           // K17 GEMM tile height (0 = by the grid fill, 128, 256)
  K17Dyn,          // K17 dynamic (claimed) tile scheduling (0 = static tile lists)
  kCount
};

long long knob(Knob k);

}  // namespace tcamd
