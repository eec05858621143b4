"""Dataset histograms (mirror of pipeline_dp/dataset_histograms): contribution
and partition statistics computed on the GPU (csrc/pdp_hist.hip)."""
from pipelinedp_amd.dataset_histograms import computing_histograms, histograms
