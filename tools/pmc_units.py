"""Summary of tools/pmc_units.sh: per (kernel, grid), averaged per dispatch,
which unit of the memory pipeline is busy.

  cu_clk      GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs): the dispatch's
              cycles at the shader clock
  ta_busy     TA_TA_BUSY summed over the 256 CUs' texture-address units, as a
              fraction of 256 x cu_clk (1.0 = every CU's TA busy every cycle)
  ta_stall_tc TA address path stalled by the L1 (TCP), same normalisation
  td_busy     TD (data return) busy fraction; td_stall_tc: TD stalled on the L1
  mfma_busy   SQ_VALU_MFMA_BUSY_CYCLES / (cu_clk x 1024): matrix pipes busy
              (4 SIMDs x 256 CUs)
  l2_req_B/clk/CU  L1 -> L2 read requests x 128 B per CU-cycle (gfx950 L1
              lines are 128 B)
  l2_hit      TCC hit fraction; rd_lat: mean L1 -> L2 read latency (cycles)
  lds_dma     LDS-DMA (buffer_load ... lds) wavefronts per dispatch
usage: python tools/pmc_units.py gpurun_out/TAG/units [name-filter]
"""
import collections
import csv
import os
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
NCU = 256
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
order = []
for p in ("p1", "p2", "p3"):
    f = f"{d}/{p}/run_counter_collection.csv"
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        name = name[-52:]
        if flt not in name:
            continue
        k = (name, r["Grid_Size"])
        if k not in agg:
            order.append(k)
        c = r["Counter_Name"]
        agg[k][(p, c)] += float(r["Counter_Value"])
        disp[k][p].add(r["Dispatch_Id"])


def per(k, p, c):
    n = max(len(disp[k][p]), 1)
    return agg[k].get((p, c), 0.0) / n


rows = []
for k in order:
    clk = per(k, "p1", "GRBM_GUI_ACTIVE") / 8
    if clk <= 0:
        continue
    clk2 = per(k, "p2", "GRBM_GUI_ACTIVE") / 8 or clk
    clk3 = per(k, "p3", "GRBM_GUI_ACTIVE") / 8 or clk
    ta = per(k, "p1", "TA_TA_BUSY_sum") / (NCU * clk)
    tas = per(k, "p1", "TA_ADDR_STALLED_BY_TC_CYCLES_sum") / (NCU * clk)
    tad = per(k, "p2", "TA_DATA_STALLED_BY_TC_CYCLES_sum") / (NCU * clk2)
    td = per(k, "p1", "TD_TD_BUSY_sum") / (NCU * clk)
    tds = per(k, "p1", "TD_TC_STALL_sum") / (NCU * clk)
    mf = per(k, "p1", "SQ_VALU_MFMA_BUSY_CYCLES") / (clk * 1024)
    wc = per(k, "p1", "SQ_WAVE_CYCLES")
    wait = per(k, "p1", "SQ_WAIT_ANY") / wc if wc else 0.0
    rq = per(k, "p2", "TCP_TCC_READ_REQ_sum")
    wq = per(k, "p2", "TCP_TCC_WRITE_REQ_sum")
    pend = per(k, "p2", "TCP_PENDING_STALL_CYCLES_sum") / (NCU * clk2)
    tcr = per(k, "p2", "TCP_TCR_TCP_STALL_CYCLES_sum") / (NCU * clk2)
    dma = per(k, "p2", "TA_BUFFER_READ_LDS_WAVEFRONTS_sum")
    hit, miss = per(k, "p3", "TCC_HIT_sum"), per(k, "p3", "TCC_MISS_sum")
    rq3 = per(k, "p3", "TCP_TCC_READ_REQ_LATENCY_sum")
    lat = rq3 / rq if rq else 0.0
    rows.append((k, clk, ta, tas, tad, td, tds, mf, wait, rq * 128 / (NCU * clk2), wq * 64 / (NCU * clk2), pend, tcr,
                 dma, hit / max(hit + miss, 1), lat))
print(f"# {d}: per dispatch; fractions of 256 CUs x the dispatch's cycles (GRBM_GUI_ACTIVE / 8)")
for (k, clk, ta, tas, tad, td, tds, mf, wait, rb, wb, pend, tcr, dma, hit, lat) in rows:
    print(f"{k[0]:52s} grid={k[1]:>7s} cu_clk={clk:8.0f} ta_busy={ta:.2f} ta_stall_tc={tas:.2f}/{tad:.2f} "
          f"td_busy={td:.2f} td_stall_tc={tds:.2f} mfma_busy={mf:.2f} wait_any={wait:.2f} "
          f"l2_rd_B/clk/CU={rb:5.1f} l2_wr_B/clk/CU={wb:5.1f} tcp_pend={pend:.2f} tcr_stall={tcr:.2f} "
          f"lds_dma={dma:9.0f} l2_hit={hit:.2f} rd_lat={lat:6.0f}")
