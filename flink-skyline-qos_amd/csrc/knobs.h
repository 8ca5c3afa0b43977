// knobs.h — environment knobs of libskyline_hip.so.
//
// Two kinds:
//  * route knobs (SKY_ENV): select between result-identical routes (prefilter on/off, brute
//    pass on/off, bounding-box pass vs round-based SFS, planned vs synchronised route, ...).
//    Every one of them is named by a test that checks the routes give the same answer.
//  * measurement knobs (SKY_MEASURE_ENV): launch-shape overrides, tracing, and the measurement
//    modes that skip work (results invalid).  They exist only in a build with -DSKY_MEASURE
//    (`make measure` -> build_measure/, used by tools/); in the product library the call is a
//    null pointer and the knob's name is not even in the binary.
#pragma once
#include <cstdlib>

#define SKY_ENV(name) std::getenv(name)
#ifdef SKY_MEASURE
#define SKY_MEASURE_ENV(name) std::getenv(name)
#else
#define SKY_MEASURE_ENV(name) (static_cast<const char *>(nullptr))
#endif
