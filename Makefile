# Top-level build: the HIP library + C++ adapter (product), the CPU oracle and
# the C++ adapter test driver (test infrastructure).
all: hip host oracle oracle_ref cpptest

hip:
	$(MAKE) -C my-lidar-graph-slam_amd/csrc

host: hip
	$(MAKE) -C my-lidar-graph-slam_amd/host

oracle:
	$(MAKE) -C oracle

# the reference's own Eigen/Boost-free sources, compiled in place (test pins)
oracle_ref:
	$(MAKE) -C oracle/ref

cpptest: host oracle
	$(MAKE) -C tests/cpp

clean:
	$(MAKE) -C my-lidar-graph-slam_amd/csrc clean
	$(MAKE) -C my-lidar-graph-slam_amd/host clean
	$(MAKE) -C oracle clean
	$(MAKE) -C oracle/ref clean
	$(MAKE) -C tests/cpp clean

.PHONY: all hip host oracle oracle_ref cpptest clean
