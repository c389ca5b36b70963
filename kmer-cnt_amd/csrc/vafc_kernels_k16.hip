// vafc_kernels_k16.hip -- instantiates the counting kernels for k = 16, 17, 18, 19.
#include "vafc_scan.h"

hipError_t vc_launch_k16(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<16>(A, grid, grid_long, st);
}
hipError_t vc_setup_k16(int lds) { return setup_k<16>(lds); }

hipError_t vc_launch_k17(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<17>(A, grid, grid_long, st);
}
hipError_t vc_setup_k17(int lds) { return setup_k<17>(lds); }

hipError_t vc_launch_k18(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<18>(A, grid, grid_long, st);
}
hipError_t vc_setup_k18(int lds) { return setup_k<18>(lds); }

hipError_t vc_launch_k19(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<19>(A, grid, grid_long, st);
}
hipError_t vc_setup_k19(int lds) { return setup_k<19>(lds); }

