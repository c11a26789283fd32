// hip-pci-bus-ids: one line per HIP device ordinal visible to this process, "<ordinal> <PCI bus id>"
// (hipDeviceGetPCIBusId, lower case). amd-gpu-discovery.sh maps rocm-smi's cards to HIP
// ordinals through it: rocm-smi numbers every card of the host, HIP only those visible
// (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES), in its own order.
#include <hip/hip_runtime.h>

#include <cctype>
#include <cstdio>

int main() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 1;
    for (int i = 0; i < n; i++) {
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, i) != hipSuccess) return 1;
        for (char* c = bus; *c; c++) *c = (char)std::tolower((unsigned char)*c);
        std::printf("%d %s\n", i, bus);
    }
    return 0;
}
