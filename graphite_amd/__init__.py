"""MI355X-native trace-driven timing engine for Graphite's emesh_hop_by_hop network model."""
