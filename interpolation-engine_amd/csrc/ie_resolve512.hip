// ie_resolve512.hip — k_resolve with 512-string tiles: ie_resolve.hip compiled a second time in
// its own namespace. Half the tiles means half the look-back hops, which pays when the evaluation
// is light and the look-back bounds the launch (the unescape command's second resolve, whose input
// is interpolation output with braces left only where they were escaped: config 4 1.77 -> 1.2 ms);
// a tile this size needs 80 KB of LDS (two workgroups per CU), which costs batches whose
// evaluation dominates (config 3: 0.95 -> 1.02 ms). ie_host.cpp picks the size per call
// (IE_OPT_TILE).
#define IE_RBLOCK 512
#define IE_RNS r512
#define IE_RESOLVE_WIDE 1
#include "ie_resolve.hip"
