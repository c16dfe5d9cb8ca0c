// mm_n07.hip — the kernels and host drivers of padded size N = 128
// (log2 N = 7), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(7)
