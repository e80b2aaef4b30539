# tools/bin/c_abi_demo: plain-C consumer of libqpsk_demod.so checked against the
# oracle (tools/c_abi_demo.c).  make -f tools/c_abi_demo.mk from the repo root.
CC ?= gcc
LIBDIR := qpsk-modulator-demodulator_amd/_build
tools/bin/c_abi_demo: tools/c_abi_demo.c include/qpsk_demod.h oracle/qpsk_oracle.h $(LIBDIR)/libqpsk_demod.so oracle/_build/liboracle.so
	mkdir -p tools/bin
	$(CC) -O2 -std=c99 -Wall -Iinclude -Ioracle -o $@ tools/c_abi_demo.c \
	  -L$(LIBDIR) -lqpsk_demod -Loracle/_build -loracle -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' \
	  -Wl,-rpath,'$$ORIGIN/../../oracle/_build'
