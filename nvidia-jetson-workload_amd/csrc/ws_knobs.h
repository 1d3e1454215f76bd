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
// march bodies step q of a multi-step launch runs behind step q-1 in the one-wave march (0:
// step q reads the row step q-1 wrote in the same body -- one dependency chain through every
// stage; 1: the two steps' stage chains are independent within a body, for one more row of
// the output ring)
#ifndef WS_DPPY_SL
#define WS_DPPY_SL 0
#endif
// WS_WAVE_STAMPS: per-workgroup start / end / placement records (tools/wave_timeline.py)
