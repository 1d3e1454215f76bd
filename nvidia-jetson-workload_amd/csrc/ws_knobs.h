// Compile-time knobs of measurement builds ONLY (tools/variant.sh NAME "-D..."): the product
// build defines none of them, and every default below is the measured choice (DESIGN.md §3.1 /
// §5 keep the numbers behind each one). Knobs measured once and settled were removed in round 4
// (consumer lag, register caps, LDS occupancy padding, row-pitch padding, cached stores, the
// scheduling barrier, the producer's prefetch distance); their results stay in DESIGN.md.
#pragma once

// LDS-DMA prefetch distance of the one-wave march, in DMA groups (0: 4 rows; by precision)
#ifndef WS_DPPY_PF
#define WS_DPPY_PF 0
#endif
// stages (bit gs - 1) taking their horizontal neighbours from LDS instead of DPP (-1: stage 1
// for one column per lane, none for pairs)
#ifndef WS_DPPY_LDSX
#define WS_DPPY_LDSX -1
#endif
// overlap schedule: a slab whose first launch's edge bands are at least WS_THIN_PCT % of its rows
// runs them as latency-critical (short chains, raised priority, reserved wave slots)
#ifndef WS_THIN_PCT
#define WS_THIN_PCT 8
#endif
// shortest edge-band chain of a thin slab's overlap, in half cones (stages per launch)
#ifndef WS_CHAIN_MIN2
#define WS_CHAIN_MIN2 2
#endif
// wave issue priority of an overlapped block's edge-band launches (0: normal)
#ifndef WS_EDGE_PRIO
#define WS_EDGE_PRIO 1
#endif
// a fused launch whose output (u, v, h, all levels) is at most WS_CACHED_MAX_MB megabytes stores it
// cached instead of nontemporal: the next launch reads it back from the Infinity Cache (0: always
// nontemporal; which precisions take it: WS_CACHED_PREC, bit 0 fp32, bit 1 fp64). C3 (48 MB):
// 0.0143 -> 0.0130 ms/step; the 8-rank C2 share (55 MB) -1 to -2 %; C2 / C4 (403 MB) stay nontemporal
#ifndef WS_CACHED_MAX_MB
#define WS_CACHED_MAX_MB 128
#endif
#ifndef WS_CACHED_PREC
#define WS_CACHED_PREC 3
#endif
// WS_WAVE_STAMPS: per-workgroup start / end / placement records (tools/wave_timeline.py)
