// CPU emulation shim for csrc/sweep.h: a few compile-time kernel sizes (the rest take the runtime-k
// instantiation, KT = 0), so the host compile stays short.
#pragma once
#define CUSTMA_SWEEP_KS(X) X(3) X(4) X(5) X(11) X(16) X(31)
