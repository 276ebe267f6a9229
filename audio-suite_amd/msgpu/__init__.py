"""msgpu: MI355X-native Microsound render engine (drop-in for main_v2.render)."""
