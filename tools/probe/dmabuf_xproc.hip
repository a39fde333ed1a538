// Probe (not product code): cross-process import of a >= 2 GiB allocation through a dmabuf fd
// fetched with pidfd_getfd.  ./dmabuf_xproc export <dir> | ./dmabuf_xproc import <dir>
#include <hip/hip_runtime.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); fflush(stdout); return 1; } } while (0)

int main(int argc, char **argv)
{
    alarm(60);
    const std::string mode = argv[1], dir = argv[2];
    const size_t total = (size_t)3 << 30, chunk = (size_t)1 << 30;
    if (mode == "export") {
        prctl(PR_SET_PTRACER, PR_SET_PTRACER_ANY, 0, 0, 0);
        char *a = nullptr;
        CK(hipMalloc(&a, total));
        for (size_t off = 0; off < total; off += chunk) CK(hipMemset(a + off, (int)(off >> 30) + 1, chunk));
        CK(hipDeviceSynchronize());
        int fd = -1;
        CK(hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)a, total, hipMemRangeHandleTypeDmaBufFd, 0));
        FILE *f = fopen((dir + "/x.tmp").c_str(), "w");
        fprintf(f, "%d %d %zu\n", (int)getpid(), fd, total);
        fclose(f);
        rename((dir + "/x.tmp").c_str(), (dir + "/x").c_str());
        printf("exported pid %d fd %d\n", (int)getpid(), fd);
        fflush(stdout);
        while (access((dir + "/done").c_str(), F_OK) != 0) usleep(10000);
        return 0;
    }
    int pid = 0, fd = 0;
    size_t sz = 0;
    while (access((dir + "/x").c_str(), F_OK) != 0) usleep(10000);
    FILE *f = fopen((dir + "/x").c_str(), "r");
    if (fscanf(f, "%d %d %zu", &pid, &fd, &sz) != 3) return 2;
    fclose(f);
    int pfd = (int)syscall(434 /* pidfd_open */, pid, 0);
    printf("pidfd_open -> %d (%s)\n", pfd, pfd < 0 ? strerror(errno) : "ok");
    int myfd = pfd < 0 ? -1 : (int)syscall(438 /* pidfd_getfd */, pfd, fd, 0);
    printf("pidfd_getfd -> %d (%s)\n", myfd, myfd < 0 ? strerror(errno) : "ok");
    fflush(stdout);
    int rc = 0;
    if (myfd >= 0) {
        hipExternalMemoryHandleDesc d = {};
        d.type = hipExternalMemoryHandleTypeOpaqueFd;
        d.handle.fd = myfd;
        d.size = sz;
        hipExternalMemory_t ext;
        hipError_t e = hipImportExternalMemory(&ext, &d);
        printf("import -> %s\n", hipGetErrorString(e));
        if (e == hipSuccess) {
            for (size_t off = 0; off < sz; off += chunk) {
                hipExternalMemoryBufferDesc bd = {};
                bd.offset = off;
                bd.size = chunk;
                void *p = nullptr;
                CK(hipExternalMemoryGetMappedBuffer(&p, ext, &bd));
                unsigned char h = 0;
                CK(hipMemcpy(&h, (char *)p + chunk - 1, 1, hipMemcpyDeviceToHost));
                printf("  chunk %zu: %d (expect %d)\n", off >> 30, h, (int)(off >> 30) + 1);
                if (h != (off >> 30) + 1) rc = 3;
            }
        } else {
            rc = 4;
        }
    } else {
        rc = 5;
    }
    fflush(stdout);
    fclose(fopen((dir + "/done").c_str(), "w"));
    return rc;
}
