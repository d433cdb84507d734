# Top-level build: the HIP library + C++ adapter (product), the CPU oracle and
# the C++ adapter test driver (test infrastructure).
all: hip host oracle cpptest

hip:
	$(MAKE) -C my-lidar-graph-slam_amd/csrc

host: hip
	$(MAKE) -C my-lidar-graph-slam_amd/host

oracle:
	$(MAKE) -C oracle

cpptest: host oracle
	$(MAKE) -C tests/cpp

clean:
	$(MAKE) -C my-lidar-graph-slam_amd/csrc clean
	$(MAKE) -C my-lidar-graph-slam_amd/host clean
	$(MAKE) -C oracle clean
	$(MAKE) -C tests/cpp clean

.PHONY: all hip host oracle cpptest clean
