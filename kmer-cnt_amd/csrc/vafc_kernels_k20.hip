// vafc_kernels_k20.hip -- instantiates the counting kernels for k = 20, 21, 22, 23.
#include "vafc_scan.h"

hipError_t vc_launch_k20(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<20>(A, grid, grid_long, st);
}
hipError_t vc_setup_k20(int lds) { return setup_k<20>(lds); }

hipError_t vc_launch_k21(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<21>(A, grid, grid_long, st);
}
hipError_t vc_setup_k21(int lds) { return setup_k<21>(lds); }

hipError_t vc_launch_k22(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<22>(A, grid, grid_long, st);
}
hipError_t vc_setup_k22(int lds) { return setup_k<22>(lds); }

hipError_t vc_launch_k23(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<23>(A, grid, grid_long, st);
}
hipError_t vc_setup_k23(int lds) { return setup_k<23>(lds); }

