# Top-level build: the HIP library (product) and the CPU oracle (test infra).
all: hip oracle

hip:
	$(MAKE) -C my-lidar-graph-slam_amd/csrc

oracle:
	$(MAKE) -C oracle

clean:
	$(MAKE) -C my-lidar-graph-slam_amd/csrc clean
	$(MAKE) -C oracle clean

.PHONY: all hip oracle clean
