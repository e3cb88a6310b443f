// Forced-include (-include) for compiling the UNMODIFIED reference file
// /root/reference/digital-filtering-c++/df/df.cpp in place.
//
// df.cpp uses a vertex array `z` (df.cpp:78, 100, 637, 724, 786) that df.hpp never
// declares (members at df.hpp:67-75), so the file does not compile as shipped.
// Unqualified lookup inside the member functions falls through class scope to the
// global namespace, so one namespace-scope vector gives those statements an object
// to bind to without touching a byte of the reference source. It is only read by
// the reference's writers (write_csv/write_tecplot/plot_rms), never by the hot path.
#include <vector>
inline std::vector<double> z;
