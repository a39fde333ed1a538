// Probe (not product code): can a sub-range of a >= 2 GiB allocation be exported as a dmabuf fd
// (hipMemGetHandleForAddressRange) and imported back (hipImportExternalMemory)?  In-process only;
// alarm() bounds a hang.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); fflush(stdout); return 1; } } while (0)

int main(int argc, char **argv)
{
    alarm(60);
    const size_t total = (size_t)(argc > 1 ? atol(argv[1]) : 3) << 30;
    const size_t chunk = (size_t)1 << 30;
    char *a = nullptr;
    CK(hipMalloc(&a, total));
    for (size_t off = 0; off < total; off += chunk) CK(hipMemset(a + off, (int)(off >> 30) + 1, chunk));
    CK(hipDeviceSynchronize());
    for (size_t off = 0; off < total; off += chunk) {
        int fd = -1;
        CK(hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)(a + (getenv("WHOLE") ? 0 : off)), getenv("WHOLE") ? total : chunk,
                                          hipMemRangeHandleTypeDmaBufFd, 0));
        printf("chunk %zu GiB: fd %d\n", off >> 30, fd); fflush(stdout);
        hipExternalMemoryHandleDesc d = {};
        d.type = hipExternalMemoryHandleTypeOpaqueFd;
        d.handle.fd = fd;
        d.size = getenv("WHOLE") ? total : chunk;
        hipExternalMemory_t ext;
        CK(hipImportExternalMemory(&ext, &d));
        hipExternalMemoryBufferDesc bd = {};
        bd.offset = getenv("WHOLE") ? off : 0;
        bd.size = chunk;
        void *p = nullptr;
        CK(hipExternalMemoryGetMappedBuffer(&p, ext, &bd));
        std::vector<unsigned char> h(4096);
        CK(hipMemcpy(h.data(), (char *)p + chunk - 4096, 4096, hipMemcpyDeviceToHost));
        printf("  mapped %p (orig %p) last byte %d expect %d\n", p, a + off, h[4095], (int)(off >> 30) + 1);
        fflush(stdout);
        CK(hipDestroyExternalMemory(ext));
    }
    printf("done\n");
    return 0;
}
