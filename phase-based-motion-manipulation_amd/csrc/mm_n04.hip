// mm_n04.hip — the kernels and host drivers of padded size N = 16
// (log2 N = 4), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(4)
